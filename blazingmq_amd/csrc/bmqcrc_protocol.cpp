// bmqcrc_protocol.cpp -- the batch callers (include/bmqcrc_protocol.h).
//
// Host walks over BlazingMQ's wire and disk formats, each followed by ONE
// batched MI355X call.  The walks gather (offset, length, expected CRC)
// arrays; all CRC arithmetic happens in bmqcrc_crc32c_batch /
// bmqcrc_crc32c_verify, which are GPU-only.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <functional>
#include <vector>

#include "../../include/bmqcrc.h"
#include "../../include/bmqcrc_protocol.h"
#include "bmqcrc_internal.h"

namespace {

inline uint32_t be32(const uint8_t* p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

inline void put_be32(uint8_t* p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

int bad_format(const char* what, uint64_t off)
{
    char buf[192];
    snprintf(buf, sizeof buf, "%s (offset %llu)", what, (unsigned long long)off);
    return bmqcrc_set_error(BMQCRC_EINVAL, buf);
}

struct Ranges {
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    std::vector<uint32_t> crc;
    std::vector<uint64_t> pos;  // CRC field position / record offset
    void push(uint64_t o, uint32_t l, uint32_t c, uint64_t p)
    {
        off.push_back(o);
        len.push_back(l);
        crc.push_back(c);
        pos.push_back(p);
    }
};

// ---------------------------------------------------------------------------
// PUT event.  EventHeader (bmqp_protocol.h:746): BE u32 F(1)|Length(31),
// u8 PV(2)|Type(6), u8 HeaderWords, u8 typeSpecific, u8 reserved.
// PutHeader (bmqp_protocol.h:1374): BE u32 Flags(4)|MessageWords(28),
// BE u32 OptionsWords(24)|CAT(3)|HeaderWords(5), BE i32 QueueId, GUID[16],
// BE u32 CRC32-C at +28.  Application data follows header + options and is
// padded to a word with 1..4 bytes equal to the count
// (ProtocolUtil::calcNumWordsAndPadding, bmqp_protocolutil.h:312).
// ---------------------------------------------------------------------------
constexpr uint32_t kEventTypePut = 2;
constexpr uint32_t kPutCrcField = 28;

int walk_put_event(const uint8_t* ev, uint64_t len, Ranges* r)
{
    if (len < 8) {
        return bad_format("PUT event shorter than its EventHeader", 0);
    }
    if ((be32(ev) & 0x7FFFFFFFu) != len) {
        return bad_format("EventHeader length differs from the event size", 0);
    }
    if ((ev[4] & 0x3Fu) != kEventTypePut) {
        return bad_format("not a PUT event", 4);
    }
    uint64_t pos = (uint64_t)ev[5] * 4;
    if (pos < 8 || pos > len) {
        return bad_format("EventHeader headerWords out of range", 5);
    }
    while (pos < len) {
        if (pos + 8 > len) {
            return bad_format("truncated PutHeader", pos);
        }
        const uint64_t msg = (uint64_t)(be32(ev + pos) & 0x0FFFFFFFu) * 4;
        const uint32_t w1 = be32(ev + pos + 4);
        const uint64_t hdr = (uint64_t)(w1 & 0x1Fu) * 4;
        const uint64_t opt = (uint64_t)(w1 >> 8) * 4;
        if (hdr < kPutCrcField + 4) {
            return bad_format("PutHeader headerWords too small for the CRC field", pos);
        }
        if (msg == 0 || pos + msg > len || hdr + opt >= msg) {
            return bad_format("PutHeader messageWords inconsistent with the event", pos);
        }
        const uint32_t pad = ev[pos + msg - 1];
        if (pad < 1 || pad > 4 || hdr + opt + pad > msg) {
            return bad_format("invalid PUT message padding", pos + msg - 1);
        }
        r->push(pos + hdr + opt, (uint32_t)(msg - hdr - opt - pad),
                be32(ev + pos + kPutCrcField), pos + kPutCrcField);
        pos += msg;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// Partition files (mqbs_filestoreprotocol.h).  FileHeader (:306): "!bmq"
// "BMQ!", u8 PV(2)|HeaderWords(6), u8 Bitness(1)|FileType(7).  Journal
// (:483): JournalFileHeader u8 headerWords, u8 recordWords (15), then 60-byte
// records; MessageRecord (:1125): type nibble in byte 0, messageOffsetDwords
// BE @32, CRC32-C BE @52, magic "*rEc" BE @56.  DATA record (:703):
// DataHeader BE u32 HW(3)|messageWords(29), BE u32 optionsWords(24)|flags(8),
// options, application data, 1..8 padding bytes equal to the count.
// ---------------------------------------------------------------------------
constexpr uint32_t kMagic1 = 0x21626D71u;  // "!bmq"
constexpr uint32_t kMagic2 = 0x424D5121u;  // "BMQ!"
constexpr uint32_t kRecordMagic = 0x2A724563u;
constexpr uint32_t kFileData = 1, kFileJournal = 2;
constexpr uint32_t kRecMessage = 1;
constexpr uint64_t kJournalRecord = 60;

int file_header_size(const uint8_t* a, uint64_t len, uint32_t want_type, uint64_t* size)
{
    if (len < 32 || be32(a) != kMagic1 || be32(a + 4) != kMagic2) {
        return bad_format("bad BlazingMQ file magic", 0);
    }
    if ((a[9] & 0x7Fu) != want_type) {
        return bad_format(want_type == kFileJournal ? "not a journal file" : "not a DATA file", 9);
    }
    *size = (uint64_t)(a[8] & 0x3Fu) * 4;
    if (*size < 32 || *size > len) {
        return bad_format("FileHeader headerWords out of range", 8);
    }
    return 0;
}

int walk_partition(const uint8_t* j, uint64_t jlen, const uint8_t* d, uint64_t dlen, Ranges* r)
{
    uint64_t fh = 0, dfh = 0;
    int rc;
    if ((rc = file_header_size(j, jlen, kFileJournal, &fh)) ||
        (rc = file_header_size(d, dlen, kFileData, &dfh))) {
        return rc;
    }
    if (fh + 2 > jlen) {
        return bad_format("truncated JournalFileHeader", fh);
    }
    if ((uint64_t)j[fh + 1] * 4 != kJournalRecord) {
        return bad_format("journal recordWords != 15", fh + 1);
    }
    const uint64_t start = fh + (uint64_t)j[fh] * 4;
    if (start > jlen) {
        return bad_format("JournalFileHeader headerWords out of range", fh);
    }
    const uint64_t nrec = (jlen - start) / kJournalRecord;
    for (uint64_t i = 0; i < nrec; ++i) {
        const uint64_t ro = start + i * kJournalRecord;
        const uint8_t* rec = j + ro;
        if (be32(rec + 56) != kRecordMagic) {
            // a pre-allocated journal is zero past the last record
            for (uint64_t b = ro; b < start + nrec * kJournalRecord; ++b) {
                if (j[b]) {
                    return bad_format("journal record with a bad magic", ro);
                }
            }
            break;
        }
        if ((rec[0] >> 4) != kRecMessage) {
            continue;
        }
        const uint64_t o = (uint64_t)be32(rec + 32) * 8;
        if (o + 8 > dlen) {
            return bad_format("DATA record offset beyond the DATA file", ro);
        }
        const uint32_t w0 = be32(d + o), w1 = be32(d + o + 4);
        const uint64_t hs = (uint64_t)(w0 >> 29) * 4;
        const uint64_t total = (uint64_t)(w0 & 0x1FFFFFFFu) * 4;
        const uint64_t opt = (uint64_t)(w1 >> 8) * 4;
        if (hs == 0 || total == 0) {
            return bad_format("DATA record with zero headerWords/messageWords", o);
        }
        if (hs + opt >= total) {
            return bad_format("DATA record header/options exceed messageWords", o);
        }
        if (o + total > dlen) {
            return bad_format("DATA record extends beyond the DATA file", o);
        }
        const uint32_t pad = d[o + total - 1];
        if (pad < 1 || pad > 8 || total < hs + opt + pad) {
            return bad_format("DATA record with invalid padding", o + total - 1);
        }
        r->push(o + hs + opt, (uint32_t)(total - hs - opt - pad), be32(rec + 52), ro);
    }
    return 0;
}

// ---------------------------------------------------------------------------
// Cluster state ledger (mqbc_clusterstateledgerprotocol.h).  File header
// (:76, 8 bytes): u8 PV(2)|HeaderWords(6), FileKey[5], reserved[2].  Record
// header (:272, 32 bytes): u8 HW(4)|RecordType(4), reserved[3], BE u32
// reserved(4)|LeaderAdvisoryWords(28), elector term, sequence number,
// timestamp.  A record is header + BER advisory + word padding + BE CRC32-C
// of everything before it; recordSize = (HW + LAW) * 4
// (mqbc_clusterstateledgerutil.h:277, appendRecord :360-417).
// ---------------------------------------------------------------------------
constexpr uint64_t kCslFileHeader = 8;
constexpr uint64_t kCslRecordHeader = 32;

void walk_csl(const uint8_t* a, uint64_t len, const uint8_t* expect_id, Ranges* r, int* walk_rc,
              uint64_t* end)
{
    *end = 0;
    if (len < kCslFileHeader) {  // log->alias of the file header fails
        *walk_rc = BMQCRC_CSL_REACHED_END_OF_LOG * 100 + BMQCRC_CSL_RECORD_ALIAS_FAILURE;
        return;
    }
    // validateFileHeader (:144-164)
    static const uint8_t kNullKey[5] = {0, 0, 0, 0, 0};
    if ((a[0] >> 6) != 1) {
        *walk_rc = BMQCRC_CSL_INVALID_PROTOCOL_VERSION;
        return;
    }
    if (memcmp(a + 1, kNullKey, 5) == 0) {
        *walk_rc = BMQCRC_CSL_INVALID_LOG_ID;
        return;
    }
    if ((a[0] & 0x3Fu) < 1) {
        *walk_rc = BMQCRC_CSL_INVALID_HEADER_WORDS;
        return;
    }
    if (expect_id && memcmp(a + 1, expect_id, 5) != 0) {
        *walk_rc = BMQCRC_CSL_INVALID_LOG_ID;
        return;
    }
    uint64_t cur = (uint64_t)(a[0] & 0x3Fu) * 4;
    while (cur + kCslRecordHeader <= len) {
        const uint8_t* h = a + cur;
        const uint32_t hw = h[0] >> 4, rt = h[0] & 0xFu;
        const uint32_t law = be32(h + 4) & 0x0FFFFFFFu;
        // validateRecordHeader (:167-185): an invalid header ends the walk cleanly
        if (hw < 1 || rt < 1 || rt > 4 || law == 0) {
            break;
        }
        const uint64_t size = ((uint64_t)hw + law) * 4;
        if (cur + size > len) {  // log->alias(&blob, recordSize, currOffset) (:293)
            *walk_rc = BMQCRC_CSL_REACHED_END_OF_LOG;
            return;
        }
        r->push(cur, (uint32_t)(size - 4), be32(a + cur + size - 4), cur);
        cur += size;
    }
    *walk_rc = 0;
    *end = cur;
}

int64_t emit(const Ranges& r, uint64_t cap, uint64_t* off, uint32_t* len, uint32_t* crc,
             uint64_t* pos)
{
    const uint64_t n = r.off.size(), k = std::min<uint64_t>(n, cap);
    if (k) {
        if (off) memcpy(off, r.off.data(), 8 * k);
        if (len) memcpy(len, r.len.data(), 4 * k);
        if (crc) memcpy(crc, r.crc.data(), 4 * k);
        if (pos) memcpy(pos, r.pos.data(), 8 * k);
    }
    return (int64_t)n;
}

// Host-pointer options: the walks always hand the GPU host buffers.
int host_opts(const bmqcrc_opts* in, bmqcrc_opts* o)
{
    if (in && in->struct_size < sizeof(bmqcrc_opts)) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "opts->struct_size too small");
    }
    if (in) {
        *o = *in;
    } else {
        memset(o, 0, sizeof *o);
        o->struct_size = sizeof *o;
    }
    if (o->flags & (BMQCRC_F_DEVICE_PTRS | BMQCRC_F_ASYNC)) {
        return bmqcrc_set_error(BMQCRC_EINVAL,
                                "protocol walks take host buffers (no DEVICE_PTRS/ASYNC)");
    }
    return 0;
}

// The walk of a verify call, run by bmqcrc_verify_host_overlapped while the
// buffer is copied to the device.
struct Overlap {
    std::function<int(Ranges*)> walk;
    Ranges r;
    bool walked = false;  // the walk succeeded
};

int overlap_prepare(void* p, const uint64_t** off, const uint32_t** len, const uint32_t** exp,
                    uint64_t* n)
{
    Overlap* o = (Overlap*)p;
    const int rc = o->walk(&o->r);
    if (rc) {
        return rc;
    }
    o->walked = true;
    *off = o->r.off.data();
    *len = o->r.len.data();
    *exp = o->r.crc.data();
    *n = o->r.off.size();
    return 0;
}

int verify_overlapped(const void* arena, uint64_t bytes, Overlap* ov, uint64_t* n_bad,
                      std::vector<uint64_t>* bad, uint64_t bad_cap, const bmqcrc_opts* opts)
{
    bmqcrc_opts o;
    int rc;
    if ((rc = host_opts(opts, &o))) {
        return rc;
    }
    return bmqcrc_verify_host_overlapped(arena, bytes, overlap_prepare, ov, n_bad, bad, bad_cap,
                                         &o);
}

}  // namespace

extern "C" {

int64_t bmqcrc_put_event_scan(const void* event, uint64_t len, uint64_t* app_off,
                              uint32_t* app_len, uint64_t* crc_pos, uint64_t cap)
{
    bmqcrc_clear_error();
    if (!event && len) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null event");
    }
    Ranges r;
    int rc = walk_put_event((const uint8_t*)event, len, &r);
    return rc ? rc : emit(r, cap, app_off, app_len, nullptr, crc_pos);
}

int64_t bmqcrc_put_event_fill_crcs(void* event, uint64_t len, const bmqcrc_opts* opts)
{
    bmqcrc_clear_error();
    if (!event && len) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null event");
    }
    bmqcrc_opts o;
    int rc;
    if ((rc = host_opts(opts, &o))) {
        return rc;
    }
    Overlap ov;  // the event's copy to the device overlaps the walk
    ov.walk = [&](Ranges* r) { return walk_put_event((const uint8_t*)event, len, r); };
    std::vector<uint32_t> out;
    if ((rc = bmqcrc_verify_host_overlapped(event, len, overlap_prepare, &ov, nullptr, nullptr, 0,
                                            &o, &out))) {
        return rc;
    }
    const Ranges& r = ov.r;
    const uint64_t n = r.off.size();
    uint8_t* ev = (uint8_t*)event;
    for (uint64_t i = 0; i < n; ++i) {
        put_be32(ev + r.pos[i], out[i]);
    }
    return (int64_t)n;
}

int bmqcrc_put_event_verify(const void* event, uint64_t len, uint64_t* n_msgs, uint64_t* n_bad,
                            uint64_t* bad_idx, uint64_t bad_cap, const bmqcrc_opts* opts)
{
    bmqcrc_clear_error();
    if ((!event && len) || !n_msgs || !n_bad || (bad_cap && !bad_idx)) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null pointer argument");
    }
    *n_msgs = *n_bad = 0;
    Overlap ov;  // the event's copy to the device overlaps the walk
    ov.walk = [&](Ranges* r) { return walk_put_event((const uint8_t*)event, len, r); };
    std::vector<uint64_t> bad;
    const int rc = verify_overlapped(event, len, &ov, n_bad, &bad, bad_cap, opts);
    *n_msgs = ov.walked ? ov.r.off.size() : 0;
    if (rc) {
        return rc;
    }
    std::copy(bad.begin(), bad.begin() + std::min<uint64_t>(*n_bad, bad.size()), bad_idx);
    return 0;
}

int64_t bmqcrc_journal_scan(const void* journal, uint64_t jlen, const void* data, uint64_t dlen,
                            uint64_t* record_off, uint64_t* app_off, uint32_t* app_len,
                            uint32_t* crc, uint64_t cap)
{
    bmqcrc_clear_error();
    if ((!journal && jlen) || (!data && dlen)) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null file buffer");
    }
    Ranges r;
    int rc = walk_partition((const uint8_t*)journal, jlen, (const uint8_t*)data, dlen, &r);
    return rc ? rc : emit(r, cap, app_off, app_len, crc, record_off);
}

int bmqcrc_recover_verify(const void* journal, uint64_t jlen, const void* data, uint64_t dlen,
                          uint64_t* n_msgs, uint64_t* n_bad, uint64_t* bad_record_off,
                          uint64_t bad_cap, const bmqcrc_opts* opts)
{
    bmqcrc_clear_error();
    if ((!journal && jlen) || (!data && dlen) || !n_msgs || !n_bad ||
        (bad_cap && !bad_record_off)) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null pointer argument");
    }
    *n_msgs = *n_bad = 0;
    // the DATA file's copy to the device overlaps the journal walk
    Overlap ov;
    ov.walk = [&](Ranges* r) {
        return walk_partition((const uint8_t*)journal, jlen, (const uint8_t*)data, dlen, r);
    };
    std::vector<uint64_t> bad;
    const int rc = verify_overlapped(data, dlen, &ov, n_bad, &bad, bad_cap, opts);
    const Ranges& r = ov.r;
    *n_msgs = ov.walked ? r.off.size() : 0;
    if (rc) {
        return rc;
    }
    const uint64_t k = std::min<uint64_t>(*n_bad, bad.size());
    for (uint64_t i = 0; i < k; ++i) {
        bad_record_off[i] = r.pos[bad[i]];
    }
    return 0;
}

int64_t bmqcrc_csl_scan(const void* log, uint64_t len, const uint8_t* expected_log_id,
                        uint64_t* rec_off, uint32_t* rec_len, uint32_t* crc, uint64_t cap,
                        int* walk_rc, uint64_t* end_offset)
{
    bmqcrc_clear_error();
    if ((!log && len) || !walk_rc || !end_offset) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null pointer argument");
    }
    Ranges r;
    walk_csl((const uint8_t*)log, len, expected_log_id, &r, walk_rc, end_offset);
    return emit(r, cap, rec_off, rec_len, crc, nullptr);
}

int bmqcrc_csl_validate(const void* log, uint64_t len, const uint8_t* expected_log_id,
                        int* csl_rc, uint64_t* offset, uint64_t* bad_record_off,
                        const bmqcrc_opts* opts)
{
    bmqcrc_clear_error();
    if ((!log && len) || !csl_rc || !offset) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null pointer argument");
    }
    int walk_rc = 0;
    uint64_t end = 0;
    Overlap ov;  // the log's copy to the device overlaps the walk
    ov.walk = [&](Ranges* r) {
        walk_csl((const uint8_t*)log, len, expected_log_id, r, &walk_rc, &end);
        return 0;
    };
    uint64_t n_bad = 0;
    std::vector<uint64_t> bad;
    const int rc = verify_overlapped(log, len, &ov, &n_bad, &bad, 1, opts);
    if (rc) {
        return rc;
    }
    const Ranges& r = ov.r;
    // The reference stops at the first failing record in log order: every
    // record gathered precedes the point where the walk itself stopped.
    if (n_bad) {
        *csl_rc = BMQCRC_CSL_INVALID_CHECKSUM;
        if (bad_record_off) {
            *bad_record_off = r.off[bad[0]];
        }
        return 0;
    }
    *csl_rc = walk_rc;
    if (walk_rc == 0) {
        *offset = end;
    }
    return 0;
}

}  // extern "C"
