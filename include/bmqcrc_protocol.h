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
 * offset.  GPU entry points return BMQCRC_ENODEV without a gfx950 device.
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

/* ---- partition recovery (mqbs_filestoreprotocol.h:306,426,483,703,1125) -- */

/* Walk a journal (FileHeader + JournalFileHeader + 60-byte records, stopping
 * at the first all-zero record) and the DATA file it points into.  For each
 * MESSAGE record i: record_off = journal offset of the record, app_off /
 * app_len = application data of its DATA record (DataHeader + options +
 * app data + 1..8 padding bytes, validated like mqbs_filestore.cpp:2495-2575),
 * crc = the CRC32C stored in the record.  Any array may be NULL. */
int64_t bmqcrc_journal_scan(const void* journal, uint64_t jlen, const void* data, uint64_t dlen,
                            uint64_t* record_off, uint64_t* app_off, uint32_t* app_len,
                            uint32_t* crc, uint64_t cap);

/* Recovery CRC check of a whole partition: one scan, one batched verify.
 * Mismatches are what the reference raises as a RECOVERY alarm and skips
 * (mqbs_filestore.cpp:2613-2624); their journal record offsets are returned
 * in ascending order (up to bad_cap). */
int bmqcrc_recover_verify(const void* journal, uint64_t jlen, const void* data, uint64_t dlen,
                          uint64_t* n_msgs, uint64_t* n_bad, uint64_t* bad_record_off,
                          uint64_t bad_cap, const bmqcrc_opts* opts);

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

/* ---- C++ spellings at the reference call sites -------------------------- */
namespace BloombergLP {
namespace bmqp {
/// Batched counterpart of the CRC step of `PutEventBuilder::packMessage`
/// (bmqp_puteventbuilder.cpp:302-320) and `PutMessageIterator` (:678), over a
/// flattened PUT event.
struct PutEventCrc32c {
    static int64_t fillAll(void* event, uint64_t len, const bmqcrc_opts* opts = 0)
    {
        return bmqcrc_put_event_fill_crcs(event, len, opts);
    }
    static int verifyAll(const void* event, uint64_t len, uint64_t* numMessages,
                         uint64_t* numBad, uint64_t* badIndices = 0, uint64_t badCap = 0,
                         const bmqcrc_opts* opts = 0)
    {
        return bmqcrc_put_event_verify(event, len, numMessages, numBad, badIndices, badCap,
                                       opts);
    }
};
}  // close namespace bmqp

namespace mqbs {
/// Batched CRC check of `FileStore::recoverMessages` (mqbs_filestore.cpp:2603).
struct FileStoreCrc32c {
    static int verifyRecovery(const void* journal, uint64_t journalLen, const void* data,
                              uint64_t dataLen, uint64_t* numMessages, uint64_t* numBad,
                              uint64_t* badRecordOffsets = 0, uint64_t badCap = 0,
                              const bmqcrc_opts* opts = 0)
    {
        return bmqcrc_recover_verify(journal, journalLen, data, dataLen, numMessages, numBad,
                                     badRecordOffsets, badCap, opts);
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
        return rc ? rc * 1000 : cslRc;
    }
};
}  // close namespace mqbc
}  // close enterprise namespace
#endif /* __cplusplus */

#endif /* BMQCRC_PROTOCOL_H */
