/* quantum.hpp -- C++ mirror of the reference's Go API on the encryption path, over the C ABI in
 * qgcm.h.  The reference is compiled Go and no Go toolchain exists in this image, so
 * the host side above the C ABI is C++ with the same package / type / function names, argument
 * meaning and error behaviour; tests/cpp/mirror_test.cpp restates crypto/crypto_test.go and
 * plugin/plugin_test.go against it.
 *
 *   quantum::common  common/common.go:16-38, 79-86   constants, StringInSlice
 *                    common/payload.go:7-45          Payload, NewTunPayload, NewSockPayload
 *                    common/mapping.go:39,54,94-103  Mapping{SupportedPlugins, AES}, MappingAES
 *   quantum::crypto  crypto/aes.go:15-83             AES (Encrypt/Decrypt/EncryptedSize/DecryptedSize), NewAES
 *                    crypto/ecdh.go:13-31            GenerateECKeyPair, GenerateSharedSecret
 *   quantum::plugin  plugin/plugin.go:14-94          Plugin, Direction, orders, Sorter (Sort), New
 *                    plugin/encryption.go:10-62      Encryption
 *                    plugin/compression.go:10-70     Compression (this repo's snappy codec)
 *                    plugin/mock.go:11-36            Mock
 *
 * Go slices become common::Slice {data, len, cap} views; Go's (value, error) pairs become
 * std::pair<T, Error> with Error::ok() == (err == nil).  Every device operation goes through
 * libqgcm (gfx950 kernels); nothing here computes AES or GHASH. */
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "qgcm.h"

namespace quantum {

// Go's `error`: empty message == nil.
struct Error {
    std::string msg;
    bool ok() const { return msg.empty(); }
};

namespace common {

constexpr int IPStart = 0;
constexpr int IPEnd = 4;
constexpr int IPLength = 4;
constexpr int PacketStart = 4;
constexpr int MaxPacketLength = 1472;
constexpr int HeaderSize = IPLength;
constexpr int OverflowSize = 35;
constexpr int MTU = MaxPacketLength - HeaderSize - OverflowSize;  // 1433

// A Go []byte view: data[0:len], capacity cap (no ownership).
struct Slice {
    uint8_t *data = nullptr;
    size_t len = 0;
    size_t cap = 0;
    // s[lo:hi], panicking (std::out_of_range) where Go would
    Slice sub(size_t lo, size_t hi) const;
    Slice from(size_t lo) const { return sub(lo, len); }
};
Slice MakeSlice(std::vector<uint8_t> &v);

struct Payload {
    Slice Raw;
    Slice Packet;
    Slice IPAddress;
    int Length = 0;
};

// common/payload.go:22-32 and :35-45.
Payload NewTunPayload(Slice raw, int packetLength);
Payload NewSockPayload(Slice raw, int packetLength);

// common/common.go:79-86.
bool StringInSlice(const std::string &a, const std::vector<std::string> &list);

}  // namespace common

namespace crypto {

constexpr int keyLength = 32;   // crypto/crypto.go:7
constexpr int SaltLength = 32;  // crypto/aes.go:15-19
constexpr int NonceSize = 12;
constexpr int Overhead = 16;

// One MI355X device's key tables (qgcm_ctx); replaces the per-process Go AEAD objects.  Key
// slots are handed out in order and never reused.
class GPUContext {
  public:
    static std::pair<std::shared_ptr<GPUContext>, Error> New(int device, uint32_t max_keys);
    ~GPUContext();
    qgcm_ctx *handle() const { return ctx_; }
    std::pair<uint32_t, Error> AllocSlot();

  private:
    explicit GPUContext(qgcm_ctx *c, uint32_t max_keys) : ctx_(c), max_(max_keys) {}
    qgcm_ctx *ctx_;
    uint32_t max_;
    uint32_t next_ = 0;
    std::mutex mu_;
};

// The process-wide device set of the reference-signature NewAES(secret, salt) below, as
// go/crypto/aes_gpu.go's Devices(): created on first use from QGCM_DEVICES ("0,1,...", default every
// visible device) and QGCM_MAX_PEERS (default 4096) as a qgcm_group, one member context per device;
// a key lives on member hash(slot) mod G.  A slot goes back to the set, its key marked unset
// (qgcm_group_clear_keys), when its AES is destroyed.
class DeviceSet {
  public:
    static std::pair<std::shared_ptr<DeviceSet>, Error> Get();
    ~DeviceSet();
    qgcm_group *handle() const { return grp_; }
    std::pair<uint32_t, Error> AllocSlot();
    void Release(uint32_t slot);

  private:
    DeviceSet(qgcm_group *g, uint32_t max_keys) : grp_(g), max_(max_keys) {}
    qgcm_group *grp_;
    uint32_t max_;
    uint32_t next_ = 0;
    std::vector<uint32_t> free_;
    std::mutex mu_;
};

// crypto/aes.go:22-26, bound to a device key slot.  Encrypt / Decrypt are virtual so that a test or
// baseline harness can run the same plugin chain over another AES-GCM (oracle/cpu_chain.cpp: the
// reference's CPU configuration with OpenSSL standing in for Go's crypto/cipher).
class AES {
  public:
    AES(std::shared_ptr<GPUContext> g, uint32_t slot) : g_(std::move(g)), ctx_(g_->handle()), slot_(slot) {}
    AES(std::shared_ptr<DeviceSet> d, qgcm_ctx *member, uint32_t slot) : d_(std::move(d)), ctx_(member), slot_(slot) {}
    virtual ~AES() {
        if (d_) d_->Release(slot_);
    }
    // one owner per key slot: a copy would give the slot back twice
    AES(const AES &) = delete;
    AES &operator=(const AES &) = delete;
    int EncryptedSize(common::Slice data) const { return (int)data.len + Overhead + NonceSize; }  // :29-31
    int DecryptedSize(common::Slice data) const { return (int)data.len - Overhead - NonceSize; }  // :34-36
    // crypto/aes.go:41-52: seals data[0:length] in place with a fresh random nonce, appends tag and
    // nonce; data needs capacity length + 28.  additional may be empty (nil).
    virtual std::pair<int, Error> Encrypt(common::Slice data, int length, common::Slice additional) const;
    // crypto/aes.go:57-62: opens data in place (nonce = last 12 B, tag the 16 before), returns
    // len - 28; on authentication failure the plaintext region is zeroed (Go 1.9 gcm.Open).
    virtual std::pair<int, Error> Decrypt(common::Slice data, common::Slice additional) const;
    uint32_t Slot() const { return slot_; }

  protected:
    AES() = default;

  private:
    std::shared_ptr<GPUContext> g_;
    std::shared_ptr<DeviceSet> d_;
    qgcm_ctx *ctx_ = nullptr;
    uint32_t slot_ = 0;
};

// crypto/aes.go:65-83: PBKDF2-HMAC-SHA512(secret, salt, 10000, 32) on the host, key schedule and
// GHASH tables on the device.  NewAES(secret, salt) is the reference's signature, on the process-wide
// DeviceSet; the other form installs the key in a given context.
std::pair<std::shared_ptr<AES>, Error> NewAES(common::Slice secret, common::Slice salt);
std::pair<std::shared_ptr<AES>, Error> NewAES(const std::shared_ptr<GPUContext> &g, common::Slice secret,
                                              common::Slice salt);

// crypto/ecdh.go:13-20 -> (pub, priv); :23-31.
std::pair<std::vector<uint8_t>, std::vector<uint8_t>> GenerateECKeyPair();
std::vector<uint8_t> GenerateSharedSecret(const std::vector<uint8_t> &pubkey, const std::vector<uint8_t> &privkey);

}  // namespace crypto

namespace common {

// common/mapping.go:39,54 -- the two fields the encryption path reads.
struct Mapping {
    std::vector<std::string> SupportedPlugins;
    std::shared_ptr<crypto::AES> AES;
};

// common/mapping.go:94-103 (ParseMapping): the peer's AES from its public key / salt and this
// node's private ones; {nullptr, nil} when the peer published no keys.
std::pair<std::shared_ptr<crypto::AES>, Error> MappingAES(const std::shared_ptr<crypto::GPUContext> &g,
                                                          const std::vector<uint8_t> &publicKey,
                                                          const std::vector<uint8_t> &publicSalt,
                                                          const std::vector<uint8_t> &privateKey,
                                                          const std::vector<uint8_t> &privateSalt);
// the same through crypto::NewAES(secret, salt), as ParseMapping calls it
std::pair<std::shared_ptr<crypto::AES>, Error> MappingAES(const std::vector<uint8_t> &publicKey,
                                                          const std::vector<uint8_t> &publicSalt,
                                                          const std::vector<uint8_t> &privateKey,
                                                          const std::vector<uint8_t> &privateSalt);

}  // namespace common

namespace plugin {

extern const char *const CompressionPlugin;  // "compression"
extern const char *const EncryptionPlugin;   // "encryption"
extern const char *const MockPlugin;         // "mock"
enum { CompressionPluginOrder = 0, EncryptionPluginOrder = 1, MockPluginOrder = 2 };

enum Direction { Incoming = 0, Outgoing = 1 };

// Apply's (*Payload, *Mapping, bool).
struct Result {
    common::Payload *payload;
    common::Mapping *mapping;
    bool ok;
};

// plugin/plugin.go:46-58.
class Plugin {
  public:
    virtual ~Plugin() = default;
    virtual Result Apply(Direction direction, common::Payload *payload, common::Mapping *mapping) = 0;
    virtual Error Close() { return {}; }
    virtual std::string Name() const = 0;
    virtual int Order() const = 0;
};

// plugin/encryption.go:10-62.
class Encryption : public Plugin {
  public:
    Result Apply(Direction direction, common::Payload *payload, common::Mapping *mapping) override;
    std::string Name() const override { return EncryptionPlugin; }
    int Order() const override { return EncryptionPluginOrder; }
};

// plugin/compression.go:10-70 (snappy block format; this repo's codec, qgcm_snappy_*).
class Compression : public Plugin {
  public:
    Result Apply(Direction direction, common::Payload *payload, common::Mapping *mapping) override;
    std::string Name() const override { return CompressionPlugin; }
    int Order() const override { return CompressionPluginOrder; }
};

// plugin/mock.go:11-36.
class Mock : public Plugin {
  public:
    Result Apply(Direction, common::Payload *payload, common::Mapping *mapping) override {
        return {payload, mapping, true};
    }
    std::string Name() const override { return MockPlugin; }
    int Order() const override { return MockPluginOrder; }
};

// sort.Sort(Sorter{Plugins: plugins}) / sort.Sort(sort.Reverse(Sorter{...})), plugin/plugin.go:63-82.
void Sort(std::vector<Plugin *> &plugins, bool reverse = false);

// plugin/plugin.go:84-94.
std::pair<std::unique_ptr<Plugin>, Error> New(const std::string &pluginType);

}  // namespace plugin
}  // namespace quantum
