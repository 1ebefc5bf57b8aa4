// C++ restatement of the reference's own tests for this path, against the C++ host mirror
// (include/quantum.hpp) over libqgcm:
//   crypto/crypto_test.go:54-101 TestAES, :133-151 TestEcdh
//   plugin/plugin_test.go:58-87 TestSorter, :89-124 TestEncryption, :126-161 TestCompression,
//                         :163-216 TestMulti, :218-232 TestMock (mapping from init() :17-28)
//   common/common_test.go:502-530 payload slicing (TestPayload)
// plus TestEncryptionTamper (Decrypt's only error, crypto/aes.go:60) and TestMappingAES
// (common/mapping.go:94-103: two peers derive the same key).
// Usage: mirror_test [TestName ...]  (no names: all).  Exit status = number of failed tests.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "quantum.hpp"

using namespace quantum;
using common::MakeSlice;
using common::Slice;

namespace {

std::string g_fail;
#define FATAL(msg)      \
    do {                \
        g_fail = (msg); \
        return;         \
    } while (0)

void randfill(uint8_t *p, size_t n) {
    size_t got = 0;
    while (got < n) {
        const ssize_t r = getrandom(p + got, n - got, 0);
        if (r > 0) got += (size_t)r;
    }
}

bool testEq(const uint8_t *a, const uint8_t *b, size_t n) { return memcmp(a, b, n) == 0; }

std::shared_ptr<crypto::GPUContext> gpu() {
    static std::shared_ptr<crypto::GPUContext> g = [] {
        auto [c, err] = crypto::GPUContext::New(0, 64);
        if (!err.ok()) fprintf(stderr, "GPUContext: %s\n", err.msg.c_str());
        return c;
    }();
    return g;
}

std::vector<uint8_t> asciiKey() {
    const char *k = "AES256Key-32Characters1234567890";
    return std::vector<uint8_t>(k, k + 32);
}

// plugin/plugin_test.go:17-28: SupportedPlugins {compression, encryption}, NewAES(key, random salt)
common::Mapping *testMapping() {
    static common::Mapping m;
    static bool init = false;
    if (!init) {
        m.SupportedPlugins = {"compression", "encryption"};
        std::vector<uint8_t> key = asciiKey(), salt(crypto::SaltLength);
        randfill(salt.data(), salt.size());
        auto [aes, err] = crypto::NewAES(gpu(), MakeSlice(key), MakeSlice(salt));
        m.AES = aes;
        init = true;
    }
    return &m;
}

// crypto/crypto_test.go TestAES, with the reference's own call: NewAES(key, salt) on the process-wide
// device set (QGCM_DEVICES, QGCM_MAX_PEERS; main() defaults them to "0,0" and 4)
void TestAES() {
    const int tagLen = 16, nonceLen = 12, bufLen = 1500, dataLen = bufLen - tagLen - nonceLen;
    std::vector<uint8_t> key = asciiKey(), salt(crypto::SaltLength);
    randfill(salt.data(), salt.size());
    auto [aes, err] = crypto::NewAES(MakeSlice(key), MakeSlice(salt));
    if (!err.ok()) FATAL("Unable to create the AES object: " + err.msg);
    std::vector<uint8_t> buf(bufLen), expected(dataLen, 1);
    memset(buf.data(), 1, dataLen);
    const Slice b = MakeSlice(buf);
    if (aes->EncryptedSize(b) != bufLen + tagLen + nonceLen) FATAL("The AES minimum size is incorrect");
    auto [length, e1] = aes->Encrypt(b, dataLen, Slice{});
    if (!e1.ok()) FATAL("Errored trying to encrypt buffer: " + e1.msg);
    if (length != aes->EncryptedSize(b.sub(0, dataLen))) FATAL("Errored determining the size of the encrypted buffer.");
    if (testEq(buf.data(), expected.data(), dataLen)) FATAL("Encrypted output matches plaintext.");
    auto [dlen, e2] = aes->Decrypt(b, Slice{});
    if (!e2.ok()) FATAL("Errored trying to decrypt buffer: " + e2.msg);
    if (dlen != dataLen) FATAL("Errored determining the size of the decrypted buffer.");
    if (!testEq(buf.data(), expected.data(), dataLen) || dataLen != aes->DecryptedSize(b))
        FATAL("Decrypted output does not match plaintext.");
}

void TestEcdh() {
    auto [pub, priv] = crypto::GenerateECKeyPair();
    if ((int)pub.size() != crypto::keyLength || (int)priv.size() != crypto::keyLength) FATAL("key lengths");
    if (pub == priv) FATAL("identical pub/priv keys");
    std::vector<uint8_t> secret = crypto::GenerateSharedSecret(pub, priv);
    if ((int)secret.size() != crypto::keyLength) FATAL("shared secret length");
    if (secret == pub || secret == priv) FATAL("secret equals a key");
    // and the exchange itself agrees from both sides
    auto [pub2, priv2] = crypto::GenerateECKeyPair();
    if (crypto::GenerateSharedSecret(pub2, priv) != crypto::GenerateSharedSecret(pub, priv2)) FATAL("X25519 disagrees");
}

void TestSorter() {
    auto [encryption, e1] = plugin::New(plugin::EncryptionPlugin);
    auto [compression, e2] = plugin::New(plugin::CompressionPlugin);
    auto [mock, e3] = plugin::New(plugin::MockPlugin);
    if (!e1.ok() || !e2.ok() || !e3.ok()) FATAL("Failed to create plugins.");
    std::vector<plugin::Plugin *> plugins = {mock.get(), encryption.get(), compression.get()};
    plugin::Sort(plugins);
    if (plugins[0]->Name() != plugin::CompressionPlugin || plugins[1]->Name() != plugin::EncryptionPlugin ||
        plugins[2]->Name() != plugin::MockPlugin)
        FATAL("Failed to properly sort the plugins");
    plugin::Sort(plugins, true);
    if (plugins[0]->Name() != plugin::MockPlugin || plugins[1]->Name() != plugin::EncryptionPlugin ||
        plugins[2]->Name() != plugin::CompressionPlugin)
        FATAL("Failed to properly reverse the plugins");
    auto [none, e4] = plugin::New("nope");
    if (none || e4.ok()) FATAL("unknown plugin accepted");
}

// one plugin, Outgoing then Incoming over a random MaxPacketLength buffer (plugin_test.go:89-161)
void roundTrip(plugin::Plugin *p, common::Mapping *mapping) {
    std::vector<uint8_t> buf(common::MaxPacketLength), expected;
    randfill(buf.data(), buf.size());
    expected = buf;
    common::Payload out = common::NewTunPayload(MakeSlice(buf), common::MTU);
    plugin::Result r = p->Apply(plugin::Outgoing, &out, mapping);
    if (!r.ok) FATAL("Failed to apply the outgoing plugin.");
    common::Payload in = common::NewSockPayload(r.payload->Raw, r.payload->Length);
    r = p->Apply(plugin::Incoming, &in, mapping);
    if (!r.ok) FATAL("Failed to apply the incoming plugin.");
    if (!testEq(expected.data(), buf.data(), common::MTU))
        FATAL("The outgoing and incoming payloads don't match after the round trip.");
    if (!p->Close().ok()) FATAL("Close failed");
}

void TestEncryption() {
    if (!gpu()) FATAL("no GPU context");
    auto [encryption, err] = plugin::New(plugin::EncryptionPlugin);
    roundTrip(encryption.get(), testMapping());
}

void TestCompression() {
    common::Mapping m;  // the compression plugin reads only SupportedPlugins
    m.SupportedPlugins = {"compression", "encryption"};
    auto [compression, err] = plugin::New(plugin::CompressionPlugin);
    roundTrip(compression.get(), &m);
    if (!g_fail.empty()) return;
    // compressible data shrinks; a corrupt stream is dropped (compression.go:37-39)
    std::vector<uint8_t> buf(common::MaxPacketLength, 'q');
    common::Payload out = common::NewTunPayload(MakeSlice(buf), common::MTU);
    plugin::Result r = compression->Apply(plugin::Outgoing, &out, &m);
    if (!r.ok || out.Length >= common::HeaderSize + 100) FATAL("compressible packet did not shrink");
    buf[common::PacketStart] = 0xff;  // varint preamble claims a huge length
    buf[common::PacketStart + 1] = 0xff;
    common::Payload in = common::NewSockPayload(MakeSlice(buf), out.Length);
    if (compression->Apply(plugin::Incoming, &in, &m).ok) FATAL("corrupt stream accepted");
}

void TestMulti() {
    if (!gpu()) FATAL("no GPU context");
    auto [encryption, e1] = plugin::New(plugin::EncryptionPlugin);
    auto [compression, e2] = plugin::New(plugin::CompressionPlugin);
    std::vector<plugin::Plugin *> plugins = {encryption.get(), compression.get()};
    plugin::Sort(plugins);
    for (int fill = 0; fill < 2; ++fill) {
        std::vector<uint8_t> buf(common::MaxPacketLength), expected;
        if (fill == 0) {
            randfill(buf.data(), buf.size());
        } else {
            for (size_t i = 0; i < buf.size(); ++i) buf[i] = "quantum packet "[i % 15];
        }
        expected = buf;
        common::Mapping *mapping = testMapping();
        common::Payload payload = common::NewTunPayload(MakeSlice(buf), common::MTU);
        common::Payload *p = &payload;
        for (plugin::Plugin *pl : plugins) {
            plugin::Result r = pl->Apply(plugin::Outgoing, p, mapping);
            if (!r.ok) FATAL("Failed to apply outgoing plugin: " + pl->Name());
            p = r.payload;
            mapping = r.mapping;
        }
        plugin::Sort(plugins, true);
        common::Payload sock = common::NewSockPayload(p->Raw, p->Length);
        p = &sock;
        for (plugin::Plugin *pl : plugins) {
            plugin::Result r = pl->Apply(plugin::Incoming, p, mapping);
            if (!r.ok) FATAL("Failed to apply incoming plugin: " + pl->Name());
            p = r.payload;
            mapping = r.mapping;
        }
        plugin::Sort(plugins);
        if (p->Length - common::HeaderSize != common::MTU)
            FATAL("The outgoing and incoming payloads have different lengths after applying all plugins.");
        // plugin_test.go:211 compares Raw[:Length-HeaderSize] with expected[:MTU]; the packet bytes
        // start at PacketStart in both, so compare those (the 4-B header is untouched)
        if (!testEq(expected.data() + common::PacketStart, p->Raw.data + common::PacketStart, common::MTU))
            FATAL("The outgoing and incoming payloads don't match after applying all plugins.");
    }
}

void TestMock() {
    auto [mock, err] = plugin::New(plugin::MockPlugin);
    plugin::Result r = mock->Apply(plugin::Outgoing, nullptr, nullptr);
    if (!r.ok || r.payload || r.mapping) FATAL("Mock Apply should always return ok.");
    if (!mock->Close().ok()) FATAL("Mock Close should always return nil.");
    if (mock->Order() != plugin::MockPluginOrder) FATAL("Mock Order should always return MockPluginOrder.");
}

void TestPayload() {
    std::vector<uint8_t> raw = {1, 2, 3, 4, 5, 6};
    common::Payload t = common::NewTunPayload(MakeSlice(raw), 2);
    if (t.IPAddress.len != 4 || t.IPAddress.data[0] != 1 || t.Packet.len != 2 || t.Packet.data[0] != 5 ||
        t.Length != 6)
        FATAL("NewTunPayload slicing");
    common::Payload s = common::NewSockPayload(MakeSlice(raw), 6);
    if (s.IPAddress.data[3] != 4 || s.Packet.len != 2 || s.Packet.data[1] != 6 || s.Length != 6)
        FATAL("NewSockPayload slicing");
    bool panicked = false;
    try {
        common::NewTunPayload(MakeSlice(raw), 3);  // raw[4:7] out of range: a Go panic
    } catch (const std::out_of_range &) {
        panicked = true;
    }
    if (!panicked) FATAL("out-of-range slice accepted");
    if (common::MTU != 1433 || common::MaxPacketLength != 1472 || common::HeaderSize != 4) FATAL("constants");
}

void TestEncryptionTamper() {
    if (!gpu()) FATAL("no GPU context");
    common::Mapping *mapping = testMapping();
    auto [enc, err] = plugin::New(plugin::EncryptionPlugin);
    std::vector<uint8_t> buf(common::MaxPacketLength);
    randfill(buf.data(), buf.size());
    common::Payload out = common::NewTunPayload(MakeSlice(buf), 1000);
    if (!enc->Apply(plugin::Outgoing, &out, mapping).ok || out.Length != 4 + 1000 + 28) FATAL("seal");
    buf[common::PacketStart + 10] ^= 0x04;
    common::Payload in = common::NewSockPayload(MakeSlice(buf), out.Length);
    if (enc->Apply(plugin::Incoming, &in, mapping).ok) FATAL("tampered packet accepted");
    for (int i = 0; i < 1000; ++i)
        if (buf[common::PacketStart + i]) FATAL("plaintext not zeroed on authentication failure");
    auto [n, e2] = mapping->AES->Decrypt(MakeSlice(buf).sub(4, 4 + 1028), Slice{});
    if (e2.ok() || n != 1000) FATAL("Decrypt must return DecryptedSize with the error");
}

void TestMappingAES() {
    if (!gpu()) FATAL("no GPU context");
    auto [apub, apriv] = crypto::GenerateECKeyPair();
    auto [aspub, aspriv] = crypto::GenerateECKeyPair();
    auto [bpub, bpriv] = crypto::GenerateECKeyPair();
    auto [bspub, bspriv] = crypto::GenerateECKeyPair();
    auto [ab, e1] = common::MappingAES(gpu(), bpub, bspub, apriv, aspriv);
    auto [ba, e2] = common::MappingAES(gpu(), apub, aspub, bpriv, bspriv);
    if (!e1.ok() || !e2.ok() || !ab || !ba || ab->Slot() == ba->Slot()) FATAL("MappingAES");
    auto [none, e3] = common::MappingAES(gpu(), {}, bspub, apriv, aspriv);
    if (none || !e3.ok()) FATAL("a peer without keys must give a nil AES and no error");
    std::vector<uint8_t> buf(1500), plain;
    randfill(buf.data(), buf.size());
    plain = buf;
    uint8_t ip[4] = {10, 99, 0, 1};
    const Slice aad{ip, 4, 4};
    auto [n, e4] = ab->Encrypt(MakeSlice(buf), 1400, aad);
    if (!e4.ok() || n != 1428) FATAL("seal with the A->B key");
    auto [m, e5] = ba->Decrypt(MakeSlice(buf).sub(0, 1428), aad);
    if (!e5.ok() || m != 1400 || !testEq(buf.data(), plain.data(), 1400)) FATAL("B cannot open A's packet");
}

// The device set hands out QGCM_MAX_PEERS slots; an AES gives its slot back when the last reference
// to it goes, so a process that makes and drops peers forever never runs out.  A key sealed through
// the device set opens through a plain context holding the same derived key (same salt, same slot
// independence: the bytes depend on the key only).
void TestNewAESSlotsRecycled() {
    std::vector<uint8_t> key = asciiKey(), salt(crypto::SaltLength);
    randfill(salt.data(), salt.size());
    std::vector<std::shared_ptr<crypto::AES>> live;
    for (int i = 0; i < 4; ++i) {
        auto [a, err] = crypto::NewAES(MakeSlice(key), MakeSlice(salt));
        if (!err.ok() || !a) FATAL("NewAES " + std::to_string(i) + ": " + err.msg);
        live.push_back(a);
    }
    {
        auto [a, err] = crypto::NewAES(MakeSlice(key), MakeSlice(salt));
        if (a || err.ok()) FATAL("a fifth live AES must fail with QGCM_MAX_PEERS=4");
    }
    std::vector<uint8_t> buf(1500), plain;
    randfill(buf.data(), buf.size());
    plain = buf;
    uint8_t ip[4] = {10, 0, 0, 7};
    const Slice aad{ip, 4, 4};
    for (int round = 0; round < 3; ++round) {
        // the slots and owners of the AES objects about to go: a Slot() kept past its AES (a batch
        // descriptor) must fail once the slot is back in the set, bytes untouched
        std::vector<std::pair<qgcm_ctx *, uint32_t>> stale;
        for (const auto &a : live)
            stale.push_back({qgcm_group_ctx(crypto::DeviceSet::Get().first->handle(),
                                            qgcm_group_shard(crypto::DeviceSet::Get().first->handle(), a->Slot())),
                             a->Slot()});
        live.clear();  // every slot back
        for (const auto &[c, s] : stale) {
            std::vector<uint8_t> z(92, 0x33), zb = z;
            if (qgcm_seal_one(c, s, z.data(), 64, nullptr, 0, nullptr) != -1 ||
                qgcm_open_one(c, s, z.data(), 92, nullptr, 0) != -1 || z != zb)
                FATAL("a released slot still seals or opens");
        }
        for (int i = 0; i < 4; ++i) {
            auto [a, err] = crypto::NewAES(MakeSlice(key), MakeSlice(salt));
            if (!err.ok() || !a) FATAL("recycled NewAES: " + err.msg);
            live.push_back(a);
        }
    }
    auto [ref, e0] = crypto::NewAES(gpu(), MakeSlice(key), MakeSlice(salt));
    if (!e0.ok() || !ref) FATAL("context NewAES: " + e0.msg);
    for (const auto &a : live) {
        auto [n, e1] = a->Encrypt(MakeSlice(buf), 1400, aad);
        if (!e1.ok() || n != 1428) FATAL("seal through the device set");
        auto [m, e2] = ref->Decrypt(MakeSlice(buf).sub(0, 1428), aad);
        if (!e2.ok() || m != 1400 || !testEq(buf.data(), plain.data(), 1400)) FATAL("context cannot open it");
    }
}

// common/mapping.go:94-103 through the reference-signature NewAES: two peers, one on the device set and
// one on a context, derive the same key
void TestMappingAESDeviceSet() {
    if (!gpu()) FATAL("no GPU context");
    auto [apub, apriv] = crypto::GenerateECKeyPair();
    auto [aspub, aspriv] = crypto::GenerateECKeyPair();
    auto [bpub, bpriv] = crypto::GenerateECKeyPair();
    auto [bspub, bspriv] = crypto::GenerateECKeyPair();
    auto [ab, e1] = common::MappingAES(bpub, bspub, apriv, aspriv);
    auto [ba, e2] = common::MappingAES(gpu(), apub, aspub, bpriv, bspriv);
    if (!e1.ok() || !e2.ok() || !ab || !ba) FATAL("MappingAES: " + e1.msg + e2.msg);
    auto [none, e3] = common::MappingAES({}, bspub, apriv, aspriv);
    if (none || !e3.ok()) FATAL("a peer without keys must give a nil AES and no error");
    std::vector<uint8_t> buf(900), plain;
    randfill(buf.data(), buf.size());
    plain = buf;
    auto [n, e4] = ab->Encrypt(MakeSlice(buf), 800, Slice{});
    if (!e4.ok() || n != 828) FATAL("seal with the A->B key");
    auto [m, e5] = ba->Decrypt(MakeSlice(buf).sub(0, 828), Slice{});
    if (!e5.ok() || m != 800 || !testEq(buf.data(), plain.data(), 800)) FATAL("B cannot open A's packet");
}

// no device set (a bad QGCM_DEVICES, or no GPU): NewAES returns the error, every time, and never a
// half-made AES
void TestNewAESNoDevices() {
    std::vector<uint8_t> key = asciiKey(), salt(crypto::SaltLength, 3);
    for (int i = 0; i < 2; ++i) {
        auto [a, err] = crypto::NewAES(MakeSlice(key), MakeSlice(salt));
        if (a || err.ok()) FATAL("NewAES must fail without a device set");
    }
}

}  // namespace

int main(int argc, char **argv) {
    setenv("QGCM_DEVICES", "0,0", 0);  // two members on one GPU: the sharding is exercised on one card
    setenv("QGCM_MAX_PEERS", "4", 0);
    const std::vector<std::pair<std::string, std::function<void()>>> tests = {
        {"TestAES", TestAES},         {"TestEcdh", TestEcdh},
        {"TestSorter", TestSorter},   {"TestEncryption", TestEncryption},
        {"TestCompression", TestCompression}, {"TestMulti", TestMulti},
        {"TestMock", TestMock},       {"TestPayload", TestPayload},
        {"TestEncryptionTamper", TestEncryptionTamper}, {"TestMappingAES", TestMappingAES},
        {"TestNewAESSlotsRecycled", TestNewAESSlotsRecycled}, {"TestMappingAESDeviceSet", TestMappingAESDeviceSet},
        {"TestNewAESNoDevices", TestNewAESNoDevices},
    };
    std::vector<std::string> want(argv + 1, argv + argc);
    int failed = 0, ran = 0;
    for (const auto &[name, fn] : tests) {
        if (!want.empty() && std::find(want.begin(), want.end(), name) == want.end()) continue;
        g_fail.clear();
        printf("=== RUN   %s\n", name.c_str());
        try {
            fn();
        } catch (const std::exception &e) {
            g_fail = std::string("panic: ") + e.what();
        }
        ++ran;
        if (g_fail.empty()) {
            printf("--- PASS: %s\n", name.c_str());
        } else {
            printf("--- FAIL: %s\n    %s\n", name.c_str(), g_fail.c_str());
            ++failed;
        }
    }
    if (ran == 0) {
        printf("no tests matched\n");
        return 1;
    }
    printf(failed ? "FAIL\n" : "PASS\n");
    return failed;
}
