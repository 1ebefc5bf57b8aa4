// quantum_host.cpp -- the C++ mirror of quantum's Go API on the encryption path (include/quantum.hpp)
// over the C ABI (include/qgcm.h).  Each function cites the Go it restates.
#include "../../include/quantum.hpp"

#include <errno.h>
#include <stdlib.h>
#include <sys/random.h>

#include <algorithm>
#include <stdexcept>

namespace quantum {

namespace common {

Slice Slice::sub(size_t lo, size_t hi) const {
    if (lo > hi || hi > cap) throw std::out_of_range("slice bounds out of range");  // a Go panic
    return Slice{data + lo, hi - lo, cap - lo};
}

Slice MakeSlice(std::vector<uint8_t> &v) { return Slice{v.data(), v.size(), v.size()}; }

// common/payload.go:22-32
Payload NewTunPayload(Slice raw, int packetLength) {
    Payload p;
    p.Raw = raw;
    p.IPAddress = raw.sub(IPStart, IPEnd);
    p.Packet = raw.sub(PacketStart, PacketStart + (size_t)packetLength);
    p.Length = HeaderSize + packetLength;
    return p;
}

// common/payload.go:35-45
Payload NewSockPayload(Slice raw, int packetLength) {
    Payload p;
    p.Raw = raw;
    p.IPAddress = raw.sub(IPStart, IPEnd);
    p.Packet = raw.sub(PacketStart, (size_t)packetLength);
    p.Length = packetLength;
    return p;
}

// common/common.go:79-86
bool StringInSlice(const std::string &a, const std::vector<std::string> &list) {
    return std::find(list.begin(), list.end(), a) != list.end();
}

}  // namespace common

namespace crypto {

std::pair<std::shared_ptr<GPUContext>, Error> GPUContext::New(int device, uint32_t max_keys) {
    char err[QGCM_ERRLEN] = {0};
    qgcm_ctx *c = qgcm_create(device, max_keys, err, (int)sizeof(err));
    if (!c) return {nullptr, Error{err[0] ? err : "qgcm_create failed"}};
    return {std::shared_ptr<GPUContext>(new GPUContext(c, max_keys)), Error{}};
}

GPUContext::~GPUContext() { qgcm_destroy(ctx_); }

std::pair<uint32_t, Error> GPUContext::AllocSlot() {
    std::lock_guard<std::mutex> g(mu_);
    if (next_ >= max_) return {0, Error{"qgcm: out of key slots"}};
    return {next_++, Error{}};
}

// crypto/aes.go:41-52.  The nonce comes from getrandom inside qgcm_seal_one (crypto/rand); an RNG
// failure is the reference's only Encrypt error, a too-small buffer is a Go panic: both -> error.
std::pair<int, Error> AES::Encrypt(common::Slice data, int length, common::Slice additional) const {
    if (length < 0 || (size_t)length + Overhead + NonceSize > data.cap)
        return {-1, Error{"crypto: buffer too small for the tag and nonce"}};
    const long n = qgcm_seal_one(ctx_, slot_, data.data, length, additional.len ? additional.data : nullptr,
                                 (uint32_t)additional.len, nullptr);
    if (n < 0) return {-1, Error{"qgcm_seal_one failed"}};
    return {(int)n, Error{}};
}

// crypto/aes.go:57-62: returns DecryptedSize(data) together with the error, as Go does.
std::pair<int, Error> AES::Decrypt(common::Slice data, common::Slice additional) const {
    const long n = qgcm_open_one(ctx_, slot_, data.data, (long)data.len,
                                 additional.len ? additional.data : nullptr, (uint32_t)additional.len);
    if (n < 0) return {DecryptedSize(data), Error{"cipher: message authentication failed"}};
    return {(int)n, Error{}};
}

std::pair<std::shared_ptr<DeviceSet>, Error> DeviceSet::Get() {
    static std::mutex mu;
    static std::shared_ptr<DeviceSet> set;
    static Error failed;
    std::lock_guard<std::mutex> lk(mu);
    if (set || !failed.ok()) return {set, failed};
    std::vector<int> devs;
    const char *spec = getenv("QGCM_DEVICES");
    if (spec && *spec) {
        for (const char *p = spec; *p;) {
            char *e;
            const long d = strtol(p, &e, 10);
            if (e == p || d < 0) {
                failed = Error{std::string("qgcm: QGCM_DEVICES=") + spec};
                return {nullptr, failed};
            }
            devs.push_back((int)d);
            p = *e == ',' ? e + 1 : e;
        }
    } else {
        for (int d = 0; d < qgcm_device_count(); ++d) devs.push_back(d);
    }
    uint32_t peers = 4096;
    if (const char *v = getenv("QGCM_MAX_PEERS"); v && *v) peers = (uint32_t)strtoul(v, nullptr, 10);
    if (devs.empty() || peers == 0 || peers > QGCM_MAX_KEYS) {
        failed = Error{"qgcm: no device set (QGCM_DEVICES / QGCM_MAX_PEERS)"};
        return {nullptr, failed};
    }
    char err[QGCM_ERRLEN] = {0};
    qgcm_group *g = qgcm_group_create(devs.data(), (int)devs.size(), peers, err, (int)sizeof(err));
    if (!g) {
        failed = Error{err[0] ? err : "qgcm_group_create failed"};
        return {nullptr, failed};
    }
    set.reset(new DeviceSet(g, peers));
    return {set, Error{}};
}

DeviceSet::~DeviceSet() { qgcm_group_destroy(grp_); }

std::pair<uint32_t, Error> DeviceSet::AllocSlot() {
    std::lock_guard<std::mutex> g(mu_);
    if (!free_.empty()) {
        const uint32_t s = free_.back();
        free_.pop_back();
        return {s, Error{}};
    }
    if (next_ >= max_) return {0, Error{"qgcm: out of key slots (QGCM_MAX_PEERS)"}};
    return {next_++, Error{}};
}

// The slot's key is marked unset before the slot is reused: a batch descriptor or a Slot() kept past the
// AES then fails its status instead of sealing under the slot's next peer's key.
void DeviceSet::Release(uint32_t slot) {
    (void)qgcm_group_clear_keys(grp_, slot, 1);
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(slot);
}

// crypto/aes.go:65-83, the reference's signature: the process-wide DeviceSet, the key on its owner
std::pair<std::shared_ptr<AES>, Error> NewAES(common::Slice secret, common::Slice salt) {
    auto [d, derr] = DeviceSet::Get();
    if (!derr.ok()) return {nullptr, derr};
    uint8_t key[QGCM_KEY_BYTES];
    if (qgcm_derive_key(secret.data, secret.len, salt.data, salt.len, key) != QGCM_OK)
        return {nullptr, Error{"qgcm_derive_key failed"}};
    auto [slot, err] = d->AllocSlot();
    if (!err.ok()) return {nullptr, err};
    qgcm_ctx *member = qgcm_group_ctx(d->handle(), qgcm_group_shard(d->handle(), slot));
    const int rc = member ? qgcm_set_key(member, slot, key) : QGCM_E_ARG;
    if (rc != QGCM_OK) {
        d->Release(slot);
        return {nullptr, Error{qgcm_strerror(rc)}};
    }
    return {std::make_shared<AES>(d, member, slot), Error{}};
}

// crypto/aes.go:65-83
std::pair<std::shared_ptr<AES>, Error> NewAES(const std::shared_ptr<GPUContext> &g, common::Slice secret,
                                              common::Slice salt) {
    uint8_t key[QGCM_KEY_BYTES];
    if (qgcm_derive_key(secret.data, secret.len, salt.data, salt.len, key) != QGCM_OK)
        return {nullptr, Error{"qgcm_derive_key failed"}};
    auto [slot, err] = g->AllocSlot();
    if (!err.ok()) return {nullptr, err};
    const int rc = qgcm_set_key(g->handle(), slot, key);
    if (rc != QGCM_OK) return {nullptr, Error{qgcm_strerror(rc)}};
    return {std::make_shared<AES>(g, slot), Error{}};
}

// crypto/ecdh.go:13-20
std::pair<std::vector<uint8_t>, std::vector<uint8_t>> GenerateECKeyPair() {
    std::vector<uint8_t> pub(keyLength), priv(keyLength);
    size_t got = 0;
    while (got < priv.size()) {  // rand.Read: its error is ignored by the reference (ecdh.go:16)
        const ssize_t r = getrandom(priv.data() + got, priv.size() - got, 0);
        if (r > 0)
            got += (size_t)r;
        else if (r < 0 && errno != EINTR)
            break;
    }
    qgcm_x25519_base(pub.data(), priv.data());
    return {pub, priv};
}

// crypto/ecdh.go:23-31 (inputs copied into 32-byte arrays: short ones zero-padded, long ones cut)
std::vector<uint8_t> GenerateSharedSecret(const std::vector<uint8_t> &pubkey, const std::vector<uint8_t> &privkey) {
    uint8_t pub[keyLength] = {0}, priv[keyLength] = {0};
    std::copy_n(pubkey.begin(), std::min<size_t>(pubkey.size(), keyLength), pub);
    std::copy_n(privkey.begin(), std::min<size_t>(privkey.size(), keyLength), priv);
    std::vector<uint8_t> secret(keyLength);
    qgcm_x25519(secret.data(), priv, pub);
    return secret;
}

}  // namespace crypto

namespace common {

// common/mapping.go:94-103
std::pair<std::shared_ptr<crypto::AES>, Error> MappingAES(const std::shared_ptr<crypto::GPUContext> &g,
                                                          const std::vector<uint8_t> &publicKey,
                                                          const std::vector<uint8_t> &publicSalt,
                                                          const std::vector<uint8_t> &privateKey,
                                                          const std::vector<uint8_t> &privateSalt) {
    if (publicKey.empty() || publicSalt.empty()) return {nullptr, Error{}};
    std::vector<uint8_t> secret = crypto::GenerateSharedSecret(publicKey, privateKey);
    std::vector<uint8_t> salt = crypto::GenerateSharedSecret(publicSalt, privateSalt);
    return crypto::NewAES(g, MakeSlice(secret), MakeSlice(salt));
}

std::pair<std::shared_ptr<crypto::AES>, Error> MappingAES(const std::vector<uint8_t> &publicKey,
                                                          const std::vector<uint8_t> &publicSalt,
                                                          const std::vector<uint8_t> &privateKey,
                                                          const std::vector<uint8_t> &privateSalt) {
    if (publicKey.empty() || publicSalt.empty()) return {nullptr, Error{}};
    std::vector<uint8_t> secret = crypto::GenerateSharedSecret(publicKey, privateKey);
    std::vector<uint8_t> salt = crypto::GenerateSharedSecret(publicSalt, privateSalt);
    return crypto::NewAES(MakeSlice(secret), MakeSlice(salt));
}

}  // namespace common

namespace plugin {

const char *const CompressionPlugin = "compression";
const char *const EncryptionPlugin = "encryption";
const char *const MockPlugin = "mock";

// plugin/encryption.go:16-40
Result Encryption::Apply(Direction direction, common::Payload *payload, common::Mapping *mapping) {
    if (!common::StringInSlice(EncryptionPlugin, mapping->SupportedPlugins)) return {payload, mapping, true};
    switch (direction) {
        case Incoming: {
            auto [length, err] = mapping->AES->Decrypt(payload->Packet, payload->IPAddress);
            if (!err.ok()) return {payload, mapping, false};
            payload->Packet = payload->Raw.sub(common::PacketStart, common::PacketStart + (size_t)length);
            payload->Length = common::HeaderSize + length;
            break;
        }
        case Outgoing: {
            auto [length, err] = mapping->AES->Encrypt(payload->Raw.from(common::PacketStart),
                                                       (int)payload->Packet.len, payload->IPAddress);
            if (!err.ok()) return {payload, mapping, false};
            payload->Packet = payload->Raw.sub(common::PacketStart, common::PacketStart + (size_t)length);
            payload->Length = common::HeaderSize + length;
            break;
        }
    }
    return {payload, mapping, true};
}

// plugin/compression.go:29-56: snappy Encode/Decode of Packet, copied into Raw[PacketStart:].
Result Compression::Apply(Direction direction, common::Payload *payload, common::Mapping *mapping) {
    if (!common::StringInSlice(CompressionPlugin, mapping->SupportedPlugins)) return {payload, mapping, true};
    const common::Slice pkt = payload->Packet;
    std::vector<uint8_t> out;
    long length = -1;
    if (direction == Incoming) {  // :35-43 decompress(); a decode error drops the packet
        const long n = qgcm_snappy_uncompressed_length(pkt.data, pkt.len);
        // a length that cannot fit Raw[PacketStart:] would make Go's re-slice panic: drop instead
        // n == 0: golang/snappy's Decode(nil, src) returns a nil slice for an empty result, and :37-39
        // drops a nil packet
        if (n <= 0 || (size_t)n > payload->Raw.cap - common::PacketStart) return {payload, mapping, false};
        out.resize((size_t)n + 1);
        length = qgcm_snappy_uncompress(pkt.data, pkt.len, out.data(), (size_t)n);
        if (length < 0) return {payload, mapping, false};
    } else {  // :44-51 compress()
        out.resize(qgcm_snappy_max_compressed_length(pkt.len));
        length = qgcm_snappy_compress(pkt.data, pkt.len, out.data(), out.size());
        if (length < 0) return {payload, mapping, false};
    }
    // copy(payload.Raw[PacketStart:], buf) copies min(len) bytes; re-slicing past cap panics in Go
    const common::Slice dst = payload->Raw.from(common::PacketStart);
    std::copy_n(out.data(), std::min<size_t>((size_t)length, dst.len), dst.data);
    payload->Packet = payload->Raw.sub(common::PacketStart, common::PacketStart + (size_t)length);
    payload->Length = common::HeaderSize + (int)length;
    return {payload, mapping, true};
}

// plugin/plugin.go:63-82 (sort.Sort is not stable; the orders are distinct)
void Sort(std::vector<Plugin *> &plugins, bool reverse) {
    std::sort(plugins.begin(), plugins.end(), [reverse](const Plugin *a, const Plugin *b) {
        return reverse ? a->Order() > b->Order() : a->Order() < b->Order();
    });
}

// plugin/plugin.go:84-94
std::pair<std::unique_ptr<Plugin>, Error> New(const std::string &pluginType) {
    if (pluginType == CompressionPlugin) return {std::make_unique<Compression>(), Error{}};
    if (pluginType == EncryptionPlugin) return {std::make_unique<Encryption>(), Error{}};
    if (pluginType == MockPlugin) return {std::make_unique<Mock>(), Error{}};
    return {nullptr, Error{"specified plugin is not supported"}};
}

}  // namespace plugin
}  // namespace quantum
