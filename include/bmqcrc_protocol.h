/* bmqcrc_protocol.h -- the batch callers of the CRC32C path (libbmqcrc.so).
 *
 * BlazingMQ computes or checks one CRC32C per message in four loops.  Each
 * entry point here walks the reference's own wire/disk format on the host
 * ("scan": CPU only, no GPU needed), then CRCs every message with ONE batched
 * MI355X call (bmqcrc_crc32c_batch / bmqcrc_crc32c_verify, include/bmqcrc.h).
 * Paths are relative to /root/reference.
 *
 *   bmqcrc_put_event_fill_crcs  bmqp::PutEventBuilder::packMessage CRC
 *                               (src/groups/bmq/bmqp/bmqp_puteventbuilder.cpp:302,320,400,413;
 *                               written to PutHeader::d_crc32c, bmqp_protocol.h:1497)
 *   bmqcrc_put_event_verify     bmqp::PutMessageIterator recompute
 *                               (bmqp_putmessageiterator.cpp:670-679)
 *   bmqcrc_recover_verify       mqbs::FileStore::recoverMessages CRC check
 *                               (src/groups/mqb/mqbs/mqbs_filestore.cpp:2495-2624)
 *   bmqcrc_csl_validate         mqbc::ClusterStateLedgerUtil::validateLog
 *                               (src/groups/mqb/mqbc/mqbc_clusterstateledgerutil.cpp:248-336)
 *
 * Buffers are host memory (an mmap'd file or an event blob flattened into one
 * buffer).  Scans return the number of messages found (which may exceed
 * `cap`; only `cap` entries are written, so cap = 0 sizes the arrays) or a
 * negative BMQCRC_E* code with bmqcrc_last_error() naming the offending
 * offset.  GPU entry points return BMQCRC_ENODEV without a gfx950 device;
 * the C++ spellings at the end of this header fall back to the host CRC.
 */
#ifndef BMQCRC_PROTOCOL_H
#define BMQCRC_PROTOCOL_H

#include <stdint.h>

#include "bmqcrc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- PUT events (bmqp_protocol.h:746 EventHeader, :1374 PutHeader) ------ */

/* Walk a PUT event: EventHeader (length must equal `len`, type e_PUT = 2)
 * then PutHeader-framed messages.  For message i: app_off/app_len = its
 * application data (after header and options, before the 1..4 padding
 * bytes) and crc_pos = byte offset of its big-endian PutHeader CRC field. */
int64_t bmqcrc_put_event_scan(const void* event, uint64_t len, uint64_t* app_off,
                              uint32_t* app_len, uint64_t* crc_pos, uint64_t cap);

/* Deferred CRC: CRC every message's application data in one batch and write
 * each result big-endian into its PutHeader.  Returns the message count. */
int64_t bmqcrc_put_event_fill_crcs(void* event, uint64_t len, const bmqcrc_opts* opts);

/* Check every PutHeader CRC against its application data in one batch.
 * *n_msgs = messages, *n_bad = mismatches, bad_idx = up to bad_cap message
 * indices in ascending order. */
int bmqcrc_put_event_verify(const void* event, uint64_t len, uint64_t* n_msgs, uint64_t* n_bad,
                            uint64_t* bad_idx, uint64_t bad_cap, const bmqcrc_opts* opts);

/* ---- partition recovery (mqbs_filestoreprotocol.h:306,426,483,703,953-1990) */

/* mqbs::FileStore::recoverMessages result codes (mqbs_filestore.cpp:1073-1091)
 * that the record selection below can produce. */
#define BMQCRC_RECOVERY_SUCCESS 0
#define BMQCRC_RECOVERY_INVALID_PRIMARY_LEASE_ID (-2)
#define BMQCRC_RECOVERY_INVALID_SEQ_NUMBER (-3)
#define BMQCRC_RECOVERY_INVALID_QUEUE_OP_RECORD (-4)
#define BMQCRC_RECOVERY_NULL_QUEUE_KEY (-5)
#define BMQCRC_RECOVERY_DUPLICATE_QUEUE_KEY (-7)
#define BMQCRC_RECOVERY_INVALID_QUEUE_KEY (-8)
#define BMQCRC_RECOVERY_INVALID_DATA_OFFSET (-11)
#define BMQCRC_RECOVERY_INVALID_SYNC_PT_SUB_TYPE (-12)
#define BMQCRC_RECOVERY_INVALID_DELETION_RECORD (-14)
#define BMQCRC_RECOVERY_INVALID_CONFIRM_RECORD (-15)
#define BMQCRC_RECOVERY_INVALID_MESSAGE_RECORD (-16)
#define BMQCRC_RECOVERY_INVALID_DATA_RECORD (-17)

/* The queues recoverMessages knows (its `withCSL` argument and
 * `queueKeyInfoMap`).  cfg == NULL or with_csl == 0: the live queues are the
 * keys of the journal's own QueueOp CREATION records (the reference's first
 * pass).  with_csl != 0: the cluster state's live queues, n_queue_keys
 * 5-byte mqbu::StorageKey values at queue_keys. */
typedef struct bmqcrc_recovery_cfg {
    uint32_t struct_size; /* sizeof(bmqcrc_recovery_cfg) */
    int32_t with_csl;
    const uint8_t* queue_keys;
    uint64_t n_queue_keys;
} bmqcrc_recovery_cfg;

/* The MESSAGE records whose payload FileStore::recoverMessages CRCs
 * (mqbs_filestore.cpp:2603-2624), selected exactly as it does: the journal
 * is bounded by its last sync point and last valid record
 * (mqbs_filestoreprotocolutil.cpp:165-289) and walked backwards twice; a
 * MESSAGE record is skipped when its GUID has a later DELETION record, its
 * queue a later whole-queue PURGE, or it precedes its queue's last
 * QueueOp DELETION -- and for skipped records the DATA file is not read.
 * Records come out in that backward order: record_off = journal offset,
 * app_off / app_len = application data of its DATA record (DataHeader +
 * options + app data + 1..8 padding bytes), crc = the stored CRC32C.
 * *recovery_rc = the reference's result (0 or BMQCRC_RECOVERY_*) and
 * *error_record_off the offending record's offset when it is not 0; the
 * records before that point are still returned (the reference had CRC'd
 * them).  Any output array may be NULL.  CPU only. */
int64_t bmqcrc_journal_scan(const void* journal, uint64_t jlen, const void* data, uint64_t dlen,
                            const bmqcrc_recovery_cfg* cfg, int* recovery_rc,
                            uint64_t* error_record_off, uint64_t* record_off, uint64_t* app_off,
                            uint32_t* app_len, uint32_t* crc, uint64_t cap);

/* The journal's bounds as JournalFileIterator computes them: *last_sync_point
 * = offset of the last well-formed SYNCPOINT record, *last_record_off = the
 * last valid record after it (0 = none; mqbs_filestoreprotocolutil.cpp:165-289).
 * Records past *last_record_off (a torn write, a pre-allocated zero tail)
 * are not part of the journal.  CPU only. */
int bmqcrc_journal_bounds(const void* journal, uint64_t jlen, uint64_t* last_sync_point,
                          uint64_t* last_record_off);

/* Recovery CRC check of a whole partition: the selection of
 * bmqcrc_journal_scan, then one batched verify on the GPU.  *n_msgs = records
 * CRC'd; mismatches are what the reference raises as a RECOVERY alarm and
 * keeps going (mqbs_filestore.cpp:2613-2624): *n_bad of them, the first
 * min(*n_bad, bad_cap) in the order the reference raises them (backward
 * journal order) in bad_record_off.  *recovery_rc / *error_record_off as
 * in bmqcrc_journal_scan. */
int bmqcrc_recover_verify(const void* journal, uint64_t jlen, const void* data, uint64_t dlen,
                          const bmqcrc_recovery_cfg* cfg, int* recovery_rc,
                          uint64_t* error_record_off, uint64_t* n_msgs, uint64_t* n_bad,
                          uint64_t* bad_record_off, uint64_t bad_cap, const bmqcrc_opts* opts);

/* ---- cluster state ledger (mqbc_clusterstateledgerprotocol.h:76,272) ------ */

/* mqbc::ClusterStateLedgerUtilRc values (mqbc_clusterstateledgerutil.h:65-124)
 * and the one mqbsi::LogOpResult a log walk can return (mqbsi_log.h:138). */
#define BMQCRC_CSL_SUCCESS 0
#define BMQCRC_CSL_INVALID_PROTOCOL_VERSION (-5)
#define BMQCRC_CSL_INVALID_LOG_ID (-6)
#define BMQCRC_CSL_INVALID_HEADER_WORDS (-7)
#define BMQCRC_CSL_INVALID_CHECKSUM (-10)
#define BMQCRC_CSL_RECORD_ALIAS_FAILURE (-13)
#define BMQCRC_CSL_REACHED_END_OF_LOG (-15)

/* Walk a ledger log like validateLog without the CRC check: validate the
 * ClusterStateFileHeader (against the 5-byte expected_log_id unless NULL),
 * then records while a whole ClusterStateRecordHeader fits; the walk stops
 * cleanly at the first invalid record header.  For record i: rec_off, and
 * rec_len = header + advisory + padding (the CRC'd bytes), crc = the trailing
 * big-endian CRC32C.  *walk_rc = the validateLog code the walk alone yields
 * (0, a file-header code, or REACHED_END_OF_LOG for a record running past
 * the end); *end_offset = where a clean walk stopped. */
int64_t bmqcrc_csl_scan(const void* log, uint64_t len, const uint8_t* expected_log_id,
                        uint64_t* rec_off, uint32_t* rec_len, uint32_t* crc, uint64_t cap,
                        int* walk_rc, uint64_t* end_offset);

/* ClusterStateLedgerUtil::validateLog with every record CRC checked in one
 * batch.  *csl_rc receives exactly the reference's result: 0 with *offset =
 * end of the valid records, INVALID_CHECKSUM for the first (lowest offset)
 * corrupt record (its offset in *bad_record_off if non-NULL), or the walk's
 * code.  The return value is a BMQCRC_E* status of the call itself. */
int bmqcrc_csl_validate(const void* log, uint64_t len, const uint8_t* expected_log_id,
                        int* csl_rc, uint64_t* offset, uint64_t* bad_record_off,
                        const bmqcrc_opts* opts);

#ifdef __cplusplus
}  /* extern "C" */

#include <vector>

/* ---- C++ spellings at the reference call sites -------------------------- */
/* The reference's calls have no error channel (bmqp_crc32c.h:240-243), so
 * these spellings never surface a GPU failure: when the batched MI355X call
 * fails for want of a GPU (BMQCRC_ENODEV, ENOMEM, EIO) they redo the same
 * walk and CRC every message on the host with the library's own SSE4.2 code
 * (bmqcrc_crc32c), bit-exact.  Format errors (BMQCRC_EINVAL) are returned.
 * Every fallback is recorded (bmqcrc_host_fallbacks, bmqcrc.h); a fault (EIO)
 * is also reported on stderr once.  The C-ABI batch entry points above stay
 * GPU-only. */
namespace BloombergLP {
namespace bmqcrc_detail {
inline bool gpuFailure(int64_t rc)
{
    if (rc == BMQCRC_ENODEV || rc == BMQCRC_ENOMEM || rc == BMQCRC_EIO) {
        bmqcrc_note_host_fallback((int32_t)rc);
        return true;
    }
    return false;
}
inline uint32_t be32(const uint8_t* p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
}  // close namespace bmqcrc_detail

namespace bmqp {
/// Batched counterpart of the CRC step of `PutEventBuilder::packMessage`
/// (bmqp_puteventbuilder.cpp:302-320) and `PutMessageIterator` (:678), over a
/// flattened PUT event.
struct PutEventCrc32c {
    static int64_t fillAll(void* event, uint64_t len, const bmqcrc_opts* opts = 0)
    {
        const int64_t rc = bmqcrc_put_event_fill_crcs(event, len, opts);
        if (!bmqcrc_detail::gpuFailure(rc)) {
            return rc;
        }
        const int64_t n = bmqcrc_put_event_scan(event, len, 0, 0, 0, 0);
        if (n <= 0) {
            return n;
        }
        std::vector<uint64_t> off(n), pos(n);
        std::vector<uint32_t> ln(n);
        bmqcrc_put_event_scan(event, len, off.data(), ln.data(), pos.data(), n);
        uint8_t* ev = static_cast<uint8_t*>(event);
        for (int64_t i = 0; i < n; ++i) {
            const uint32_t c = bmqcrc_crc32c(ev + off[i], ln[i], 0);
            ev[pos[i]] = (uint8_t)(c >> 24);
            ev[pos[i] + 1] = (uint8_t)(c >> 16);
            ev[pos[i] + 2] = (uint8_t)(c >> 8);
            ev[pos[i] + 3] = (uint8_t)c;
        }
        return n;
    }
    static int verifyAll(const void* event, uint64_t len, uint64_t* numMessages,
                         uint64_t* numBad, uint64_t* badIndices = 0, uint64_t badCap = 0,
                         const bmqcrc_opts* opts = 0)
    {
        const int rc = bmqcrc_put_event_verify(event, len, numMessages, numBad, badIndices,
                                               badCap, opts);
        if (!bmqcrc_detail::gpuFailure(rc)) {
            return rc;
        }
        const int64_t n = bmqcrc_put_event_scan(event, len, 0, 0, 0, 0);
        if (n < 0) {
            return (int)n;
        }
        std::vector<uint64_t> off(n), pos(n);
        std::vector<uint32_t> ln(n);
        bmqcrc_put_event_scan(event, len, off.data(), ln.data(), pos.data(), n);
        const uint8_t* ev = static_cast<const uint8_t*>(event);
        uint64_t bad = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (bmqcrc_crc32c(ev + off[i], ln[i], 0) != bmqcrc_detail::be32(ev + pos[i])) {
                if (bad < badCap) {
                    badIndices[bad] = (uint64_t)i;
                }
                ++bad;
            }
        }
        *numMessages = (uint64_t)n;
        *numBad = bad;
        return 0;
    }
};
}  // close namespace bmqp

namespace mqbs {
/// Batched CRC check of `FileStore::recoverMessages` (mqbs_filestore.cpp:2603),
/// over the same records the reference CRCs (see bmqcrc_recover_verify).
struct FileStoreCrc32c {
    static int verifyRecovery(const void* journal, uint64_t journalLen, const void* data,
                              uint64_t dataLen, int* recoveryRc, uint64_t* numMessages,
                              uint64_t* numBad, uint64_t* badRecordOffsets = 0,
                              uint64_t badCap = 0, const bmqcrc_recovery_cfg* cfg = 0,
                              const bmqcrc_opts* opts = 0, uint64_t* errorRecordOffset = 0)
    {
        const int rc = bmqcrc_recover_verify(journal, journalLen, data, dataLen, cfg, recoveryRc,
                                             errorRecordOffset, numMessages, numBad,
                                             badRecordOffsets, badCap, opts);
        if (!bmqcrc_detail::gpuFailure(rc)) {
            return rc;
        }
        const int64_t n = bmqcrc_journal_scan(journal, journalLen, data, dataLen, cfg,
                                              recoveryRc, errorRecordOffset, 0, 0, 0, 0, 0);
        if (n < 0) {
            return (int)n;
        }
        std::vector<uint64_t> rec(n), off(n);
        std::vector<uint32_t> ln(n), crc(n);
        bmqcrc_journal_scan(journal, journalLen, data, dataLen, cfg, recoveryRc,
                            errorRecordOffset, rec.data(), off.data(), ln.data(), crc.data(), n);
        const uint8_t* d = static_cast<const uint8_t*>(data);
        uint64_t bad = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (bmqcrc_crc32c(d + off[i], ln[i], 0) != crc[i]) {
                if (bad < badCap) {
                    badRecordOffsets[bad] = rec[i];
                }
                ++bad;
            }
        }
        *numMessages = (uint64_t)n;
        *numBad = bad;
        return 0;
    }
};
}  // close namespace mqbs

namespace mqbc {
/// `ClusterStateLedgerUtil::validateLog` (mqbc_clusterstateledgerutil.cpp:248)
/// over a mapped log: returns the reference's rc, sets `*offset` on success.
struct ClusterStateLedgerCrc32c {
    static int validateLog(uint64_t* offset, const void* log, uint64_t len,
                           const uint8_t* expectedLogId = 0, const bmqcrc_opts* opts = 0)
    {
        int cslRc = 0;
        const int rc = bmqcrc_csl_validate(log, len, expectedLogId, &cslRc, offset, 0, opts);
        if (!bmqcrc_detail::gpuFailure(rc)) {
            return rc ? rc * 1000 : cslRc;
        }
        int walkRc = 0;
        uint64_t end = 0;
        const int64_t n = bmqcrc_csl_scan(log, len, expectedLogId, 0, 0, 0, 0, &walkRc, &end);
        if (n < 0) {
            return (int)n * 1000;
        }
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> ln(n), crc(n);
        bmqcrc_csl_scan(log, len, expectedLogId, off.data(), ln.data(), crc.data(), n, &walkRc,
                        &end);
        const uint8_t* a = static_cast<const uint8_t*>(log);
        for (int64_t i = 0; i < n; ++i) {  // the first corrupt record in log order
            if (bmqcrc_crc32c(a + off[i], ln[i], 0) != crc[i]) {
                return BMQCRC_CSL_INVALID_CHECKSUM;
            }
        }
        if (walkRc == 0) {
            *offset = end;
        }
        return walkRc;
    }
};
}  // close namespace mqbc
}  // close enterprise namespace
#endif /* __cplusplus */

#endif /* BMQCRC_PROTOCOL_H */
