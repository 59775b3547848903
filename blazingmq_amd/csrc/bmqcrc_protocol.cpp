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
#include <functional>
#include <string>
#include <unordered_map>
#include <unordered_set>
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
// records.  Every record starts with a RecordHeader (:1014): BE u16
// type(4)|flags(12), BE u16 + BE u32 sequence number (48 bits), BE u32
// primary lease id, BE u64 timestamp; and ends with the magic "*rEc" @56.
// Record bodies (byte offsets in the 60-byte record):
//   MessageRecord   (:1125) queueKey[5] @22, messageOffsetDwords @32,
//                           GUID[16] @36, CRC32-C @52
//   ConfirmRecord   (:1339) queueKey @22, appKey @27, GUID @32
//   DeletionRecord  (:1518) queueKey @23, GUID @28
//   QueueOpRecord   (:1694) queueKey @22, appKey @27, BE i32 QueueOpType @32
//   JournalOpRecord (:1953) syncPointType u8 @23, BE i32 JournalOpType @24,
//                           sequence number @28/@32, primary lease id @40,
//                           dataFileOffsetDwords @44
// DATA record (:703): DataHeader BE u32 HW(3)|messageWords(29), BE u32
// optionsWords(24)|flags(8), options, application data, 1..8 padding bytes
// equal to the count.
// ---------------------------------------------------------------------------
constexpr uint32_t kMagic1 = 0x21626D71u;  // "!bmq"
constexpr uint32_t kMagic2 = 0x424D5121u;  // "BMQ!"
constexpr uint32_t kRecordMagic = 0x2A724563u;
constexpr uint32_t kFileData = 1, kFileJournal = 2;
constexpr uint32_t kRecUndefined = 0, kRecMessage = 1, kRecConfirm = 2, kRecDeletion = 3,
                   kRecQueueOp = 4, kRecJournalOp = 5;                 // RecordType (:953)
constexpr int32_t kOpUndefined = 0, kOpPurge = 1, kOpCreation = 2, kOpDeletion = 3,
                  kOpAddition = 4;                                     // QueueOpType (:1630)
constexpr int32_t kJournalOpSyncPoint = 2;                             // JournalOpType (:1841)
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

struct RecHeader {
    uint32_t type;
    uint32_t lease;
    uint64_t seq;
};

inline RecHeader rec_header(const uint8_t* r)
{
    RecHeader h;
    h.type = r[0] >> 4;
    h.seq = ((uint64_t)(((uint32_t)r[2] << 8) | r[3]) << 32) | be32(r + 4);
    h.lease = be32(r + 8);
    return h;
}

// mqbu::StorageKey (5 bytes) as an integer; the null key is 0.
inline uint64_t key5(const uint8_t* p)
{
    return ((uint64_t)p[0] << 32) | ((uint64_t)p[1] << 24) | ((uint64_t)p[2] << 16) |
           ((uint64_t)p[3] << 8) | p[4];
}

struct Guid {
    uint64_t hi, lo;
    bool operator==(const Guid& o) const { return hi == o.hi && lo == o.lo; }
    bool unset() const { return hi == 0 && lo == 0; }  // bmqt::MessageGUID::isUnset
};

inline Guid guid_at(const uint8_t* p)
{
    Guid g{0, 0};
    for (int i = 0; i < 8; ++i) {
        g.hi = (g.hi << 8) | p[i];
        g.lo = (g.lo << 8) | p[8 + i];
    }
    return g;
}

struct GuidHash {
    size_t operator()(const Guid& g) const
    {
        return (size_t)(g.hi * 0x9E3779B97F4A7C15ull ^ (g.lo + 0x632BE59BD9B4E019ull));
    }
};

// FileStoreProtocolUtil::lastJournalSyncPoint (mqbs_filestoreprotocolutil.cpp:165-228):
// scan backwards for the last well-formed SYNCPOINT JournalOp record; 0 = none.
uint64_t last_sync_point_of(const uint8_t* j, uint64_t jlen, uint64_t start)
{
    if (jlen <= start) {
        return 0;
    }
    const uint64_t nrec = (jlen - start) / kJournalRecord;
    for (uint64_t i = 1; i <= nrec; ++i) {
        const uint64_t pos = start + (nrec - i) * kJournalRecord;
        const uint8_t* r = j + pos;
        const RecHeader h = rec_header(r);
        if (h.type != kRecJournalOp || (int32_t)be32(r + 24) != kJournalOpSyncPoint ||
            h.lease == 0 || h.seq == 0 || be32(r + 56) != kRecordMagic) {
            continue;
        }
        return pos;
    }
    return 0;
}

// FileStoreProtocolUtil::lastJournalRecord (:230-289): from the last sync
// point, forward until a record with an undefined type or a bad magic; the
// record before it is the last one.  0 = the journal holds no record.
uint64_t last_record(const uint8_t* j, uint64_t jlen, uint64_t start, uint64_t lsp)
{
    if (jlen <= start) {
        return 0;
    }
    uint64_t cur = lsp ? lsp + kJournalRecord : start;
    uint64_t prev = lsp;
    while (cur + kJournalRecord <= jlen) {
        const uint8_t* r = j + cur;
        if ((r[0] >> 4) == kRecUndefined || be32(r + kJournalRecord - 4) != kRecordMagic) {
            return prev;
        }
        prev = cur;
        cur += kJournalRecord;
    }
    return prev;
}

// What FileStore::recoverMessages knows about the partition's queues: with
// CSL the cluster state's queue keys, without it the keys of the journal's
// QueueOp CREATION records (its first pass).
struct QueueView {
    bool with_csl = false;
    std::unordered_set<uint64_t> keys;  // queueKeyInfoMap
};

struct RecoveryResult {
    int rc = BMQCRC_RECOVERY_SUCCESS;
    uint64_t error_record = 0;  // journal offset of the record that failed recovery
};

// mqbs::FileStore::recoverMessages (mqbs_filestore.cpp:1045-2666) reduced to
// the decisions that select which MESSAGE records get their payload CRC'd
// (:2603-2624) and the record checks that abort recovery on the way.  Both
// passes iterate the journal backwards from its last record
// (JournalFileIterator in reverse mode, mqbs_journalfileiterator.cpp:38-281),
// stopping at the first record with an undefined type, a zero lease id or
// sequence number, or a bad magic.  The write head is the last record's PSN
// (the FSM workflow, mqbs_filestore.cpp:497-517).  Ranges come out in that
// backward order, which is the order the reference raises its alarms in.
//
// Not restated: the QLIST file (the partition is read qlist-unaware), the
// in-memory record map, purges of one appKey (they do not skip the message's
// CRC) and the legacy multi-node truncation to the last sync point.
int walk_recovery(const uint8_t* j, uint64_t jlen, const uint8_t* d, uint64_t dlen,
                  QueueView* qv, Ranges* r, RecoveryResult* res)
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
    if (j[fh] == 0) {  // JournalFileIterator::reset rc_CORRUPT_JOURNAL_HEADER
        return bad_format("JournalFileHeader headerWords is zero", fh);
    }
    if ((uint64_t)j[fh + 1] * 4 != kJournalRecord) {
        return bad_format("journal recordWords != 15", fh + 1);
    }
    const uint64_t start = fh + (uint64_t)j[fh] * 4;
    if (start > jlen) {
        return bad_format("JournalFileHeader headerWords out of range", fh);
    }
    const uint64_t last = last_record(j, jlen, start, last_sync_point_of(j, jlen, start));
    if (last == 0) {
        return 0;  // no records: nothing to recover
    }
    // Records of the backward iteration: last, last - 60, ..., start.
    auto valid = [&](uint64_t pos) {
        const uint8_t* rec = j + pos;
        const RecHeader h = rec_header(rec);
        return h.type != kRecUndefined && h.lease != 0 && h.seq != 0 &&
               be32(rec + kJournalRecord - 4) == kRecordMagic;
    };
    auto fail_at = [&](int code, uint64_t pos) {
        res->rc = code;
        res->error_record = pos;
        return 0;
    };
    // Partitions hold few queues and a walk meets the same key in long runs:
    // remember the last answer instead of hashing every record.
    uint64_t live_key = ~0ull;
    bool live_ans = false;
    auto live = [&](uint64_t key) {
        if (key != live_key) {
            live_key = key;
            live_ans = qv->keys.count(key) != 0;
        }
        return live_ans;
    };

    // ---- first pass (:1120-1453): deleted queues, queues alive without CSL,
    // the first sync point's offset.
    std::unordered_map<uint64_t, uint64_t> deleted_queue;  // queueKey -> DELETION offset
    std::unordered_map<uint64_t, uint64_t> deleted_app;    // appKey -> DELETION offset
    uint64_t first_sync = 0;
    for (uint64_t pos = last + kJournalRecord; pos >= start + kJournalRecord;) {
        pos -= kJournalRecord;
        if (!valid(pos)) {
            break;
        }
        const uint8_t* rec = j + pos;
        const uint32_t type = rec[0] >> 4;
        if (type == kRecJournalOp) {
            first_sync = pos;
            continue;
        }
        if (type != kRecQueueOp) {
            continue;
        }
        const int32_t op = (int32_t)be32(rec + 32);
        const uint64_t qkey = key5(rec + 22), akey = key5(rec + 27);
        if (op == kOpUndefined) {
            return fail_at(BMQCRC_RECOVERY_INVALID_QUEUE_OP_RECORD, pos);
        }
        if (qkey == 0) {
            return fail_at(BMQCRC_RECOVERY_NULL_QUEUE_KEY, pos);
        }
        if (op == kOpDeletion) {
            if (qv->with_csl && akey == 0 && live(qkey)) {
                return fail_at(BMQCRC_RECOVERY_INVALID_DELETION_RECORD, pos);
            }
            // the last DELETION of a key (the first one met backwards) counts
            (akey == 0 ? deleted_queue : deleted_app).emplace(akey == 0 ? qkey : akey, pos);
        } else if (op == kOpPurge) {
            continue;
        } else if (op == kOpAddition || op == kOpCreation) {
            if (deleted_queue.count(qkey)) {
                continue;
            }
            if (qv->with_csl) {
                if (!live(qkey)) {
                    return fail_at(BMQCRC_RECOVERY_INVALID_QUEUE_KEY, pos);
                }
            } else if (op == kOpAddition) {
                if (live(qkey)) {  // a CREATION met earlier backwards: two live queues
                    return fail_at(BMQCRC_RECOVERY_DUPLICATE_QUEUE_KEY, pos);
                }
            } else if (live_key = ~0ull, !qv->keys.insert(qkey).second) {
                return fail_at(BMQCRC_RECOVERY_DUPLICATE_QUEUE_KEY, pos);
            }
        }
        // any other QueueOpType: alarmed and skipped (:1443-1451)
    }

    // ---- second pass (:1490-2646)
    std::unordered_set<Guid, GuidHash> deleted_guids;
    std::unordered_set<uint64_t> purged_queues;
    const RecHeader head = rec_header(j + last);
    uint32_t lease = head.lease;
    uint64_t seq = head.seq + 1;
    auto before_queue_deletion = [&](uint64_t qkey, uint64_t pos) {
        if (deleted_queue.empty()) {
            return false;
        }
        auto it = deleted_queue.find(qkey);
        return it != deleted_queue.end() && pos < it->second;
    };
    for (uint64_t pos = last + kJournalRecord; pos >= start + kJournalRecord;) {
        pos -= kJournalRecord;
        if (!valid(pos)) {
            break;
        }
        const uint8_t* rec = j + pos;
        const RecHeader h = rec_header(rec);
        // PSN checks (:1495-1555)
        if (h.lease > lease) {
            return fail_at(BMQCRC_RECOVERY_INVALID_PRIMARY_LEASE_ID, pos);
        }
        if (h.lease == lease) {
            const bool bad = pos >= first_sync ? h.seq != seq - 1 : h.seq > seq - 1;
            if (bad) {
                return fail_at(BMQCRC_RECOVERY_INVALID_SEQ_NUMBER, pos);
            }
        }
        lease = h.lease;
        seq = h.seq;

        if (h.type == kRecJournalOp) {  // :1571-1716
            const uint64_t sp_seq = ((uint64_t)be32(rec + 28) << 32) | be32(rec + 32);
            const uint32_t sp_lease = be32(rec + 40);
            const uint64_t data_off = (uint64_t)be32(rec + 44) * 8;
            if (rec[23] == 0) {
                return fail_at(BMQCRC_RECOVERY_INVALID_SYNC_PT_SUB_TYPE, pos);
            }
            if (data_off == 0 || dlen < data_off) {
                return fail_at(BMQCRC_RECOVERY_INVALID_DATA_OFFSET, pos);
            }
            if (sp_lease == 0) {
                return fail_at(BMQCRC_RECOVERY_INVALID_PRIMARY_LEASE_ID, pos);
            }
            if (sp_seq == 0) {
                return fail_at(BMQCRC_RECOVERY_INVALID_SEQ_NUMBER, pos);
            }
            if (sp_lease > lease) {
                return fail_at(BMQCRC_RECOVERY_INVALID_PRIMARY_LEASE_ID, pos);
            }
            if (sp_lease == lease && sp_seq != seq) {
                return fail_at(BMQCRC_RECOVERY_INVALID_SEQ_NUMBER, pos);
            }
        } else if (h.type == kRecQueueOp) {  // :1717-2233
            const uint64_t qkey = key5(rec + 22), akey = key5(rec + 27);
            const int32_t op = (int32_t)be32(rec + 32);
            if (before_queue_deletion(qkey, pos)) {
                continue;  // :1778-1787, :2003-2013
            }
            if (op == kOpAddition && !qv->with_csl && !live(qkey)) {
                // an ADDITION whose CREATION the first pass did not see (:2018-2030)
                return fail_at(BMQCRC_RECOVERY_INVALID_QUEUE_KEY, pos);
            }
            if (op != kOpPurge || !live(qkey)) {
                continue;  // only a whole-queue purge of a live queue skips messages
            }
            if (akey == 0) {
                purged_queues.insert(qkey);
            }
        } else if (h.type == kRecDeletion) {  // :2234-2305
            const uint64_t qkey = key5(rec + 23);
            const Guid g = guid_at(rec + 28);
            if (g.unset() || qkey == 0) {
                return fail_at(BMQCRC_RECOVERY_INVALID_DELETION_RECORD, pos);
            }
            if (before_queue_deletion(qkey, pos) || purged_queues.count(qkey)) {
                continue;
            }
            deleted_guids.insert(g);  // kept even for an unknown queue (alarmed)
        } else if (h.type == kRecConfirm) {  // :2306-2389
            if (guid_at(rec + 32).unset() || key5(rec + 22) == 0) {
                return fail_at(BMQCRC_RECOVERY_INVALID_CONFIRM_RECORD, pos);
            }
        } else if (h.type == kRecMessage) {  // :2390-2645
            const uint64_t qkey = key5(rec + 22);
            const Guid g = guid_at(rec + 36);
            if (g.unset() || qkey == 0) {
                return fail_at(BMQCRC_RECOVERY_INVALID_MESSAGE_RECORD, pos);
            }
            const uint64_t o = (uint64_t)be32(rec + 32) * 8;
            if (o == 0 || o > dlen) {
                return fail_at(BMQCRC_RECOVERY_INVALID_DATA_OFFSET, pos);
            }
            if (before_queue_deletion(qkey, pos) ||
                (!purged_queues.empty() && purged_queues.count(qkey))) {
                continue;  // the DATA file is never touched for these (:2390-2393)
            }
            if (!deleted_guids.empty()) {
                auto del = deleted_guids.find(g);
                if (del != deleted_guids.end()) {
                    deleted_guids.erase(del);
                    continue;
                }
            }
            // DATA record checks (:2494-2575).  Where the reference would read
            // past the end of the DATA file, the record is invalid here.
            if (o + 8 > dlen) {
                return fail_at(BMQCRC_RECOVERY_INVALID_DATA_RECORD, pos);
            }
            const uint32_t w0 = be32(d + o), w1 = be32(d + o + 4);
            const uint64_t hs = (uint64_t)(w0 >> 29) * 4;
            const uint64_t total = (uint64_t)(w0 & 0x1FFFFFFFu) * 4;
            const uint64_t opt = (uint64_t)(w1 >> 8) * 4;
            if (hs == 0 || total == 0 || hs + opt >= total || o + total > dlen) {
                return fail_at(BMQCRC_RECOVERY_INVALID_DATA_RECORD, pos);
            }
            const uint32_t pad = d[o + total - 1];
            if (pad < 1 || pad > 8 || total < hs + opt + pad) {
                return fail_at(BMQCRC_RECOVERY_INVALID_DATA_RECORD, pos);
            }
            if (!live(qkey)) {
                return fail_at(BMQCRC_RECOVERY_INVALID_QUEUE_KEY, pos);
            }
            r->push(o + hs + opt, (uint32_t)(total - hs - opt - pad), be32(rec + 52), pos);
        }
    }
    return 0;
}

int recovery_view(const bmqcrc_recovery_cfg* cfg, QueueView* qv)
{
    if (!cfg) {
        return 0;
    }
    if (cfg->struct_size < sizeof(bmqcrc_recovery_cfg)) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "cfg->struct_size too small");
    }
    qv->with_csl = cfg->with_csl != 0;
    if (qv->with_csl) {
        if (cfg->n_queue_keys && !cfg->queue_keys) {
            return bmqcrc_set_error(BMQCRC_EINVAL, "null queue_keys");
        }
        for (uint64_t i = 0; i < cfg->n_queue_keys; ++i) {
            qv->keys.insert(key5(cfg->queue_keys + 5 * i));
        }
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
                      std::vector<uint64_t>* bad, uint64_t bad_cap, const bmqcrc_opts* opts,
                      uint64_t* n_written)
{
    bmqcrc_opts o;
    int rc;
    if ((rc = host_opts(opts, &o))) {
        return rc;
    }
    return bmqcrc_verify_host_overlapped(arena, bytes, overlap_prepare, ov, n_bad, bad, bad_cap,
                                         &o, nullptr, n_written);
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
    uint64_t n_written = 0;
    const int rc = verify_overlapped(event, len, &ov, n_bad, &bad, bad_cap, opts, &n_written);
    *n_msgs = ov.walked ? ov.r.off.size() : 0;
    if (rc) {
        return rc;
    }
    std::copy(bad.begin(), bad.begin() + n_written, bad_idx);
    return 0;
}

int64_t bmqcrc_journal_scan(const void* journal, uint64_t jlen, const void* data, uint64_t dlen,
                            const bmqcrc_recovery_cfg* cfg, int* recovery_rc,
                            uint64_t* error_record_off, uint64_t* record_off, uint64_t* app_off,
                            uint32_t* app_len, uint32_t* crc, uint64_t cap)
{
    bmqcrc_clear_error();
    if ((!journal && jlen) || (!data && dlen) || !recovery_rc) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null pointer argument");
    }
    QueueView qv;
    Ranges r;
    RecoveryResult res;
    int rc = recovery_view(cfg, &qv);
    if (!rc) {
        rc = walk_recovery((const uint8_t*)journal, jlen, (const uint8_t*)data, dlen, &qv, &r,
                           &res);
    }
    if (rc) {
        return rc;
    }
    *recovery_rc = res.rc;
    if (error_record_off) {
        *error_record_off = res.error_record;
    }
    return emit(r, cap, app_off, app_len, crc, record_off);
}

int bmqcrc_journal_bounds(const void* journal, uint64_t jlen, uint64_t* last_sync_point,
                          uint64_t* last_record_off)
{
    bmqcrc_clear_error();
    if ((!journal && jlen) || !last_sync_point || !last_record_off) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null pointer argument");
    }
    const uint8_t* j = (const uint8_t*)journal;
    uint64_t fh = 0;
    int rc = file_header_size(j, jlen, kFileJournal, &fh);
    if (rc) {
        return rc;
    }
    if (fh + 2 > jlen || j[fh] == 0 || fh + (uint64_t)j[fh] * 4 > jlen) {
        return bad_format("bad JournalFileHeader", fh);
    }
    if ((uint64_t)j[fh + 1] * 4 != kJournalRecord) {
        return bad_format("journal recordWords != 15", fh + 1);
    }
    const uint64_t start = fh + (uint64_t)j[fh] * 4;
    *last_sync_point = last_sync_point_of(j, jlen, start);
    *last_record_off = last_record(j, jlen, start, *last_sync_point);
    return 0;
}

int bmqcrc_recover_verify(const void* journal, uint64_t jlen, const void* data, uint64_t dlen,
                          const bmqcrc_recovery_cfg* cfg, int* recovery_rc,
                          uint64_t* error_record_off, uint64_t* n_msgs, uint64_t* n_bad,
                          uint64_t* bad_record_off, uint64_t bad_cap, const bmqcrc_opts* opts)
{
    bmqcrc_clear_error();
    if ((!journal && jlen) || (!data && dlen) || !recovery_rc || !n_msgs || !n_bad ||
        (bad_cap && !bad_record_off)) {
        return bmqcrc_set_error(BMQCRC_EINVAL, "null pointer argument");
    }
    *n_msgs = *n_bad = 0;
    *recovery_rc = 0;
    QueueView qv;
    RecoveryResult res;
    int rc = recovery_view(cfg, &qv);
    if (rc) {
        return rc;
    }
    // the DATA file's copy to the device overlaps the journal walk
    Overlap ov;
    ov.walk = [&](Ranges* r) {
        return walk_recovery((const uint8_t*)journal, jlen, (const uint8_t*)data, dlen, &qv, r,
                             &res);
    };
    std::vector<uint64_t> bad;
    uint64_t n_written = 0;
    rc = verify_overlapped(data, dlen, &ov, n_bad, &bad, bad_cap, opts, &n_written);
    const Ranges& r = ov.r;
    *n_msgs = ov.walked ? r.off.size() : 0;
    if (ov.walked) {
        *recovery_rc = res.rc;
        if (error_record_off) {
            *error_record_off = res.error_record;
        }
    }
    if (rc) {
        return rc;
    }
    for (uint64_t i = 0; i < n_written; ++i) {
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
    const int rc = verify_overlapped(log, len, &ov, &n_bad, &bad, 1, opts, nullptr);
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
