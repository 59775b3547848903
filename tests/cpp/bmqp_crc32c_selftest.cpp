// bmqp_crc32c_selftest.cpp -- the reference's component test plan for
// bmqp::Crc32c (/root/reference/src/groups/bmq/bmqp/bmqp_crc32c.t.cpp),
// re-run against the drop-in include/bmqp_crc32c.h.  Expected values are the
// reference's own golden constants.
//
//   bmqp_selftest            CPU cases 1-5, 7, 8 (+ fuzz property)
//   bmqp_selftest gpu        requires the MI355X for the batch paths
#include "bmqcrc_protocol.h"
#include "bmqp_crc32c.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <thread>
#include <vector>

using BloombergLP::bdlbb::Blob;
using BloombergLP::bdlbb::BlobBuffer;
using BloombergLP::bmqp::Crc32c;

static int g_fail = 0;
#define CHECK_EQ(a, b)                                                                     \
    do {                                                                                   \
        unsigned long long a_ = (a), b_ = (b);                                             \
        if (a_ != b_) {                                                                    \
            fprintf(stderr, "%s:%d: %s = %#llx != %#llx\n", __FILE__, __LINE__, #a, a_, b_); \
            ++g_fail;                                                                      \
        }                                                                                  \
    } while (0)

struct V {
    const char* buf;
    unsigned crc;
};
static const V k_DATA[] = {{"", 0},
                           {"DYB|O", 0},
                           {"0", 0x629E1AE0},
                           {"1", 0x90F599E3},
                           {"2", 0x83A56A17},
                           {"~", 0x8F9DB87B},
                           {"22", 0x47B26CF9},
                           {"fa", 0x8B9F1387},
                           {"t0-", 0x77E2D1A9},
                           {"34v}", 0x031AD8A7},
                           {"shaii", 0xB0638FB5},
                           {"3jf-_3", 0xE186B745},
                           {"bonjour", 0x156088D2},
                           {"vbPHbvtB", 0x12AAFAA6},
                           {"aoDicgezd", 0xBF5E01C8},
                           {"123456789", 0xe3069283},
                           {"gaaXsSP1al", 0xC4E61D23},
                           {"2Wm9bbNDehd", 0x54A11873},
                           {"GamS0NJhAl8y", 0x0044AC66}};
static const size_t k_N = sizeof(k_DATA) / sizeof(*k_DATA);

static void test1_breathing()
{
    CHECK_EQ(Crc32c::calculate("12345678", 8), 0x6087809Au);
    CHECK_EQ(Crc32c::calculate(0, 0), 0u);
    CHECK_EQ(Crc32c::calculate("12345678", 0), 0u);
    CHECK_EQ(Crc32c::calculate("12345678", 0, 0x6087809A), 0x6087809Au);
    const unsigned pre = Crc32c::calculate("12345678", 3);
    CHECK_EQ(Crc32c::calculate("12345678" + 3, 5, pre), 0x6087809Au);
}

static void test2_3_buffer_and_misaligned()
{
    alignas(16) char scratch[1024];
    for (size_t i = 0; i < k_N; ++i) {
        const unsigned len = (unsigned)strlen(k_DATA[i].buf);
        CHECK_EQ(Crc32c::calculate(k_DATA[i].buf, len), k_DATA[i].crc);
        for (unsigned mis = 1; mis < 16; ++mis) {
            memset(scratch, 'X', mis);
            memcpy(scratch + mis, k_DATA[i].buf, len);
            CHECK_EQ(Crc32c::calculate(scratch + mis, len), k_DATA[i].crc);
        }
    }
}

static void test4_previous_crc()
{
    struct T {
        const char* buf;
        unsigned pre;
        unsigned crc;
    } d[] = {{"", 0, 0},
             {"DYB|O--", 5, 0xD1436CCE},
             {"0sef", 1, 0x50588062},
             {"13", 1, 0x813E4763},
             {"2s34faw", 1, 0xED5E0C1C},
             {"~ahaer", 1, 0x45F10742},
             {"22aasd", 2, 0x22B28122},
             {"faghar", 2, 0xD9253928},
             {"t0-aavk", 3, 0x8A752D3F},
             {"34v}acv", 4, 0xC36C7D1D},
             {"shaiig5bg", 5, 0x9E26CF81},
             {"123456789", 9, 0xe3069283},
             {"3jf-_3adfg", 6, 0xEDA627B3},
             {"bonjour421h", 7, 0xD23EF1DF},
             {"vbPHbvtB45gga", 8, 0xFCC29260},
             {"aoDicgezd==7h", 9, 0x171D042A},
             {"gaaXsSP1aldsafad", 10, 0xFD5078EF},
             {"2Wm9bbNDehd32qf", 11, 0x9F7277C6},
             {"GamS0NJhAl8yw3th", 12, 0x6033D909}};
    for (const T& t : d) {
        const unsigned len = (unsigned)strlen(t.buf);
        unsigned c = Crc32c::calculate(t.buf, t.pre);
        c = Crc32c::calculate(t.buf + t.pre, len - t.pre, c);
        CHECK_EQ(c, t.crc);
        CHECK_EQ(Crc32c::calculate(t.buf, 0, c), c);
        CHECK_EQ(Crc32c::calculate(0, 0, c), c);
    }
}

static void test5_multithreaded()
{
    enum { k_NUM_PAYLOADS = 10000, k_NUM_THREADS = 10 };
    std::mt19937 rng(5);
    std::vector<std::string> payloads;
    for (int i = 0; i < k_NUM_PAYLOADS; ++i) {
        std::string s(i + 1, '\0');
        for (auto& ch : s) {
            ch = (char)rng();
        }
        payloads.push_back(s);
    }
    std::vector<unsigned> serial;
    for (auto& p : payloads) {
        serial.push_back(Crc32c::calculate(p.data(), (unsigned)p.size()));
    }
    std::vector<std::vector<unsigned>> res(k_NUM_THREADS);
    std::vector<std::thread> th;
    for (int t = 0; t < k_NUM_THREADS; ++t) {
        th.emplace_back([&, t]() {
            for (auto& p : payloads) {
                res[t].push_back(Crc32c::calculate(p.data(), (unsigned)p.size()));
            }
        });
    }
    for (auto& t : th) {
        t.join();
    }
    for (int t = 0; t < k_NUM_THREADS; ++t) {
        for (int j = 0; j < k_NUM_PAYLOADS; ++j) {
            CHECK_EQ(res[t][j], serial[j]);
        }
    }
}

static std::string sentence()
{
    std::string s =
        "This will be put in a blob buffer of typical"
        " size, and then we will test the crc32c calculation"
        " (blob version) with only one blob buffer to ensure"
        " that the logic of the loop works even for one blob"
        " buffer. Moreover, append some lines bellow to increase"
        " the size of this buffer.";
    return s + std::string(550, '#');
}

static void test7_8_blob()
{
    Blob empty;
    CHECK_EQ(Crc32c::calculate(empty), Crc32c::k_NULL_CRC32C);
    CHECK_EQ(Crc32c::calculate(empty, 0xA0EA6901), 0xA0EA6901u);

    char one[] = "one", two[] = "two", three[] = "three";
    Blob b;
    b.appendDataBuffer(BlobBuffer(one, 3));
    b.appendDataBuffer(BlobBuffer(two, 3));
    b.appendDataBuffer(BlobBuffer(three, 5));
    CHECK_EQ(Crc32c::calculate(b), 0xA0EA6901u);

    Blob b1, b2;
    b1.appendDataBuffer(BlobBuffer(one, 3));
    b2.appendDataBuffer(BlobBuffer(two, 3));
    b2.appendDataBuffer(BlobBuffer(three, 5));
    CHECK_EQ(Crc32c::calculate(b2, Crc32c::calculate(b1)), 0xA0EA6901u);

    std::string s = sentence();
    Blob one_buf;
    one_buf.appendDataBuffer(BlobBuffer(&s[0], (int)s.size()));
    CHECK_EQ(Crc32c::calculate(one_buf), 0xD86F726Eu);

    // lastDataBufferLength() trims the last buffer only
    std::string padded = s + "garbage";
    Blob trimmed;
    trimmed.appendDataBuffer(BlobBuffer(&padded[0], (int)padded.size()));
    trimmed.setLastDataBufferLength((int)s.size());
    CHECK_EQ(Crc32c::calculate(trimmed), 0xD86F726Eu);
}

static void fuzz_blob_equals_raw()
{
    // s_bmqfuzz_bmqp_crc32c.fuzz.cpp:29-55: raw CRC == Blob CRC for any
    // buffer size in 1..256 and any seed.
    std::mt19937 rng(77);
    for (int it = 0; it < 2000; ++it) {
        const int size = 1 + (int)(rng() % 256);
        std::string data(size, '\0');
        for (auto& ch : data) {
            ch = (char)rng();
        }
        const unsigned seed = rng();
        Blob blob;
        int pos = 0;
        while (pos < size) {
            const int take = 1 + (int)(rng() % (size - pos));
            blob.appendDataBuffer(BlobBuffer(&data[pos], take));
            pos += take;
        }
        CHECK_EQ(Crc32c::calculate(blob, seed), Crc32c::calculate(data.data(), size, seed));
    }
}

// ---- protocol walks (include/bmqcrc_protocol.h) --------------------------
static void put_be32(std::string* s, size_t at, unsigned v)
{
    (*s)[at] = (char)(v >> 24);
    (*s)[at + 1] = (char)(v >> 16);
    (*s)[at + 2] = (char)(v >> 8);
    (*s)[at + 3] = (char)v;
}

static unsigned get_be32(const std::string& s, size_t at)
{
    const unsigned char* p = (const unsigned char*)s.data() + at;
    return ((unsigned)p[0] << 24) | ((unsigned)p[1] << 16) | ((unsigned)p[2] << 8) | p[3];
}

// PUT event: EventHeader + (PutHeader(36) + app data + 1..4 padding) each,
// CRC fields left zero (the deferred-CRC builder state).
static std::string put_event(const std::vector<std::string>& apps)
{
    std::string ev(8, '\0');
    for (const std::string& a : apps) {
        const int pad = 4 - (int)(a.size() % 4);
        const unsigned words = (unsigned)((36 + a.size() + pad) / 4);
        std::string h(36, '\0');
        put_be32(&h, 0, words);
        put_be32(&h, 4, 9);  // headerWords
        ev += h + a + std::string(pad, (char)pad);
    }
    put_be32(&ev, 0, (unsigned)ev.size());
    ev[4] = (char)((1 << 6) | 2);  // PV 1, e_PUT
    ev[5] = 2;
    return ev;
}

// Cluster state ledger: file header + records (header 32 + advisory + word
// padding + BE CRC), appendRecord's layout.
static std::string csl_record(const std::string& adv, int type)
{
    std::string r(32, '\0');
    r += adv;
    const int pad = 4 - (int)(r.size() % 4);
    r += std::string(pad, (char)pad);
    r[0] = (char)((8 << 4) | type);
    put_be32(&r, 4, (unsigned)((r.size() + 4) / 4 - 8));
    const unsigned crc = Crc32c::calculate(r.data(), (unsigned)r.size());
    r += std::string(4, '\0');
    put_be32(&r, r.size() - 4, crc);
    return r;
}

static void protocol_scans(std::vector<std::string>* apps, std::string* ev, std::string* log)
{
    std::mt19937 rng(21);
    for (int i = 0; i < 300; ++i) {
        apps->emplace_back(rng() % 3000, '\0');
        for (auto& ch : apps->back()) {
            ch = (char)rng();
        }
    }
    *ev = put_event(*apps);
    std::vector<unsigned long long> off(apps->size()), pos(apps->size());
    std::vector<unsigned> len(apps->size());
    CHECK_EQ(bmqcrc_put_event_scan(ev->data(), ev->size(), 0, 0, 0, 0), apps->size());
    CHECK_EQ(bmqcrc_put_event_scan(ev->data(), ev->size(), (uint64_t*)off.data(), len.data(),
                                   (uint64_t*)pos.data(), off.size()),
             apps->size());
    for (size_t i = 0; i < apps->size(); ++i) {
        CHECK_EQ(len[i], (*apps)[i].size());
        CHECK_EQ(memcmp(ev->data() + off[i], (*apps)[i].data(), len[i]), 0);
        CHECK_EQ(pos[i] + 8, off[i]);  // CRC field at PutHeader+28, app data at +36
    }
    std::string bad = *ev;
    bad[4] = 3;  // not a PUT event
    CHECK_EQ(bmqcrc_put_event_scan(bad.data(), bad.size(), 0, 0, 0, 0), BMQCRC_EINVAL);

    const unsigned char key[5] = {1, 2, 3, 4, 5};
    *log = std::string(1, (char)((1 << 6) | 2)) + std::string((const char*)key, 5) +
           std::string(2, '\0');
    for (int i = 0; i < 40; ++i) {
        *log += csl_record(std::string(1 + rng() % 500, (char)('a' + i % 26)), 1 + i % 4);
    }
    int walk_rc = 1;
    uint64_t end = 0;
    CHECK_EQ(bmqcrc_csl_scan(log->data(), log->size(), key, 0, 0, 0, 0, &walk_rc, &end), 40);
    CHECK_EQ(walk_rc, 0);
    CHECK_EQ(end, log->size());
}

// The C++ call-site spellings: on the GPU, or on the host when there is none.
static void protocol_spellings(const std::vector<std::string>& apps, std::string ev,
                               std::string log)
{
    using namespace BloombergLP;
    CHECK_EQ(bmqp::PutEventCrc32c::fillAll(&ev[0], ev.size()), apps.size());
    std::vector<unsigned long long> off(apps.size());
    std::vector<unsigned> len(apps.size());
    bmqcrc_put_event_scan(ev.data(), ev.size(), (uint64_t*)off.data(), len.data(), 0,
                          off.size());
    for (size_t i = 0; i < apps.size(); ++i) {
        CHECK_EQ(get_be32(ev, off[i] - 8), Crc32c::calculate(apps[i].data(),
                                                             (unsigned)apps[i].size()));
    }
    uint64_t n = 0, nbad = 0, idx[4] = {0, 0, 0, 0};
    CHECK_EQ(bmqp::PutEventCrc32c::verifyAll(ev.data(), ev.size(), &n, &nbad, idx, 4), 0);
    CHECK_EQ(nbad, 0u);
    ev[off[7]] ^= 1;
    CHECK_EQ(bmqp::PutEventCrc32c::verifyAll(ev.data(), ev.size(), &n, &nbad, idx, 4), 0);
    CHECK_EQ(n, apps.size());
    CHECK_EQ(nbad, 1u);
    CHECK_EQ(idx[0], 7u);

    const unsigned char key[5] = {1, 2, 3, 4, 5};
    uint64_t offset = 0;
    CHECK_EQ(mqbc::ClusterStateLedgerCrc32c::validateLog(&offset, log.data(), log.size(), key),
             0);
    CHECK_EQ(offset, log.size());
    log[8 + 32] ^= 1;  // first advisory byte of the first record
    CHECK_EQ(mqbc::ClusterStateLedgerCrc32c::validateLog(&offset, log.data(), log.size(), key),
             BMQCRC_CSL_INVALID_CHECKSUM);
}

// The reference's on-disk fixture (bmqstoragetool integration data, copied
// to tests/golden/): two MESSAGE records whose app data "hello world" has
// CRC32-C 3381945770 (detail_result.txt:15,53), journal offsets 224 and 644.
static bool read_file(const std::string& path, std::string* out)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        return false;
    }
    out->assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return true;
}

static bool fixture(std::string* journal, std::string* data)
{
    const char* dir = getenv("BMQCRC_GOLDEN_DIR");
    if (!dir) {
        return false;
    }
    const bool ok = read_file(std::string(dir) + "/test.bmq_journal", journal) &&
                    read_file(std::string(dir) + "/test.bmq_data", data);
    if (!ok) {
        fprintf(stderr, "fixture: cannot read %s\n", dir);
        ++g_fail;
    }
    return ok;
}

static void recovery_scan(const std::string& j, const std::string& d)
{
    // FileStore::recoverMessages CRCs only the second message: the first
    // one's GUID has a DELETION record at offset 404 (mqbs_filestore.cpp:2481).
    uint64_t rec[4], off[4], err = 7;
    uint32_t len[4], crc[4];
    int rrc = 1;
    CHECK_EQ(bmqcrc_journal_scan(j.data(), j.size(), d.data(), d.size(), 0, &rrc, &err, rec, off,
                                 len, crc, 4),
             1);
    CHECK_EQ(rrc, 0);
    CHECK_EQ(rec[0], 644u);
    CHECK_EQ(len[0], 11u);
    CHECK_EQ(crc[0], 3381945770u);
    CHECK_EQ(memcmp(d.data() + off[0], "hello world", 11), 0);
    CHECK_EQ(Crc32c::calculate(d.data() + off[0], len[0]), 3381945770u);
}

// The C++ spelling: on the GPU, or on the host when there is none.
static void recovery_verify(const std::string& j, std::string d)
{
    using namespace BloombergLP;
    uint64_t n = 0, bad = 0, where[2] = {0, 0};
    int rrc = 1;
    CHECK_EQ(mqbs::FileStoreCrc32c::verifyRecovery(j.data(), j.size(), d.data(), d.size(), &rrc,
                                                   &n, &bad, where, 2),
             0);
    CHECK_EQ(rrc, 0);
    CHECK_EQ(n, 1u);
    CHECK_EQ(bad, 0u);
    d[52 + 4] ^= 0x20;  // the deleted message's payload: never CRC'd, no alarm
    CHECK_EQ(mqbs::FileStoreCrc32c::verifyRecovery(j.data(), j.size(), d.data(), d.size(), &rrc,
                                                   &n, &bad, where, 2),
             0);
    CHECK_EQ(bad, 0u);
    d[76 + 4] ^= 0x20;  // the live message's payload: "hello World"
    CHECK_EQ(mqbs::FileStoreCrc32c::verifyRecovery(j.data(), j.size(), d.data(), d.size(), &rrc,
                                                   &n, &bad, where, 2),
             0);
    CHECK_EQ(bad, 1u);
    CHECK_EQ(where[0], 644u);
}

// calculateBatch overloads: on the GPU, or on the host when there is none.
static void batch_overloads()
{
    std::string arena;
    std::vector<unsigned long long> off;
    std::vector<unsigned> len, exp;
    for (size_t i = 0; i < k_N; ++i) {
        off.push_back(arena.size());
        len.push_back((unsigned)strlen(k_DATA[i].buf));
        exp.push_back(k_DATA[i].crc);
        arena += k_DATA[i].buf;
    }
    std::string s = sentence();
    off.push_back(arena.size());
    len.push_back((unsigned)s.size());
    exp.push_back(0xD86F726E);
    arena += s;
    std::vector<unsigned> got(off.size());
    const int rc = Crc32c::calculateBatch(arena.data(), arena.size(), off.data(), len.data(), 0,
                                          got.data(), off.size());
    CHECK_EQ(rc, 0);
    for (size_t i = 0; i < got.size(); ++i) {
        CHECK_EQ(got[i], exp[i]);
    }

    // batched Blob overload vs the scalar Blob overload
    std::mt19937 rng(99);
    std::vector<std::string> store;
    store.reserve(4096);
    std::vector<Blob> blobs(300);
    std::vector<unsigned> seeds(blobs.size()), bexp(blobs.size()), bgot(blobs.size());
    for (size_t b = 0; b < blobs.size(); ++b) {
        const int nb = (int)(rng() % 9);
        for (int i = 0; i < nb; ++i) {
            store.emplace_back(rng() % 5000, '\0');
            for (auto& ch : store.back()) {
                ch = (char)rng();
            }
            blobs[b].appendDataBuffer(BlobBuffer(&store.back()[0], (int)store.back().size()));
        }
        seeds[b] = (rng() & 1) ? rng() : 0;
        bexp[b] = Crc32c::calculate(blobs[b], seeds[b]);
    }
    CHECK_EQ(Crc32c::calculateBatch(blobs.data(), (unsigned)blobs.size(), seeds.data(),
                                    bgot.data()),
             0);
    for (size_t b = 0; b < blobs.size(); ++b) {
        CHECK_EQ(bgot[b], bexp[b]);
    }
}

int main(int argc, char** argv)
{
    test1_breathing();
    test2_3_buffer_and_misaligned();
    test4_previous_crc();
    test5_multithreaded();
    test7_8_blob();
    fuzz_blob_equals_raw();
    std::vector<std::string> apps;
    std::string ev, log;
    protocol_scans(&apps, &ev, &log);
    std::string journal, data;
    const bool have_fixture = fixture(&journal, &data);
    if (have_fixture) {
        recovery_scan(journal, data);
    }
    const bool gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    if (gpu && bmqcrc_device_count() <= 0) {
        fprintf(stderr, "gpu: no device\n");
        ++g_fail;
    }
    if (!gpu && bmqcrc_device_count() == 0) {
        // without a GPU the C-ABI batch path refuses loudly, never falls back
        uint32_t out = 0;
        uint64_t o = 0;
        uint32_t l = 1;
        CHECK_EQ((unsigned)bmqcrc_crc32c_batch("x", 1, &o, &l, 0, &out, 1, 0),
                 (unsigned)BMQCRC_ENODEV);
        std::string ev2 = ev;
        CHECK_EQ((unsigned)bmqcrc_put_event_fill_crcs(&ev2[0], ev2.size(), 0),
                 (unsigned)BMQCRC_ENODEV);
    }
    // ... while the C++ spellings at the reference call sites give the same
    // bit-exact answers on either path
    batch_overloads();
    protocol_spellings(apps, ev, log);
    if (have_fixture) {
        recovery_verify(journal, data);
    }
    // every host fallback is recorded: none with a GPU, one per spelling without
    int32_t last_rc = 0;
    const uint64_t fallbacks = bmqcrc_host_fallbacks(&last_rc);
    if (bmqcrc_device_count() > 0) {
        CHECK_EQ((unsigned)fallbacks, 0u);
    } else {
        CHECK_EQ((unsigned)(fallbacks > 0), 1u);
        CHECK_EQ((unsigned)last_rc, (unsigned)BMQCRC_ENODEV);
    }
    printf("%s: %d failure(s)\n", g_fail ? "FAIL" : "PASS", g_fail);
    return g_fail ? 1 : 0;
}
