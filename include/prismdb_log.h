/*
 * prismdb_log.h -- batched log (WAL / MANIFEST) record checking, host side.
 *
 * SURVEY 8(f) #4.  PrismDB's logs use LevelDB's record format
 * (db/log_format.h): 32 KiB blocks of physical records
 *     crc[4] | length[2] | type[1] | payload[length]
 * with crc = Mask(crc32c(type || payload)) (db/log_writer.cc:94-97).
 * log::Reader (db/log_reader.cc) checks one record at a time.  The batched
 * form splits it in three:
 *
 *   1. leveldb_log_scan     (host)   lists every physical record the reader can
 *                                    reach, trusting the length fields;
 *   2. leveldb_crc32c_batch[_host]   with PRISMDB_CRC32C_LOG_HEADER checks all
 *                                    of them at once on the device
 *                                    (span = record + 6, len = 1 + length);
 *   3. leveldb_log_replay   (host)   runs log::Reader::ReadRecord's state
 *                                    machine over the scan and the device's
 *                                    mismatch flags and returns exactly the
 *                                    records and Reporter::Corruption calls
 *                                    the reference reader produces.
 *
 * Records after a checksum mismatch in the same block are scanned and checked
 * speculatively; the replay drops them as the reference does
 * (db/log_reader.cc:248-258: the rest of the block is discarded).
 */
#ifndef PRISMDB_LOG_H_
#define PRISMDB_LOG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LEVELDB_LOG_BLOCK_SIZE 32768 /* db/log_format.h kBlockSize */
#define LEVELDB_LOG_HEADER_SIZE 7    /* db/log_format.h kHeaderSize */

/* Reporter::Corruption reasons (db/log_reader.cc), as codes.  Codes >= 256
 * are "unknown record type %u" for the raw type byte code - 256; the text
 * prints it as the reader does (the byte goes through a signed char,
 * db/log_reader.cc:222, so 0x80..0xFF print as 4294967168..4294967295) --
 * see leveldb_log_reason(). */
#define LEVELDB_LOG_CHECKSUM_MISMATCH 1   /* "checksum mismatch"                     :256 */
#define LEVELDB_LOG_BAD_RECORD_LENGTH 2   /* "bad record length"                     :228 */
#define LEVELDB_LOG_PARTIAL_NO_END_1 3    /* "partial record without end(1)"         :100 */
#define LEVELDB_LOG_PARTIAL_NO_END_2 4    /* "partial record without end(2)"         :116 */
#define LEVELDB_LOG_MISSING_START_1 5     /* "missing start of fragmented record(1)" :126 */
#define LEVELDB_LOG_MISSING_START_2 6     /* "missing start of fragmented record(2)" :135 */
#define LEVELDB_LOG_ERROR_IN_MIDDLE 7     /* "error in middle of record"             :156 */
#define LEVELDB_LOG_UNKNOWN_TYPE_BASE 256 /* "unknown record type %u"                :164 */

#define LEVELDB_LOG_EINVAL (-1)
#define LEVELDB_LOG_ECAPACITY (-11)

/*
 * Physical records reachable by log::Reader(file, checksum, initial_offset):
 * header offsets rec_off[i] and payload lengths rec_len[i], ascending.  Writes
 * min(total, cap) entries; *n_out = total; returns LEVELDB_LOG_ECAPACITY when
 * cap was too small (size / 7 + 1 always suffices).
 */
int leveldb_log_scan(const void* file, size_t size, uint64_t initial_offset, uint64_t* rec_off,
                     uint32_t* rec_len, size_t cap, size_t* n_out);

/* Output arrays of leveldb_log_replay (caller-owned; capacities in *_cap). */
typedef struct leveldb_log_replay_out {
  /* logical records, in ReadRecord order */
  uint64_t* record_offset; /* Reader::LastRecordOffset() after the record */
  uint32_t* record_first;  /* first fragment of the record in fragment[] */
  uint32_t* record_nfrag;  /* number of fragments (1 for a kFullType record) */
  size_t record_cap, n_records;
  /* fragments: indices into the scanned physical records; the bytes are
   * file[rec_off[k] + 7, rec_off[k] + 7 + rec_len[k]) */
  uint32_t* fragment;
  size_t fragment_cap, n_fragments;
  /* Reporter::Corruption(bytes, reason) calls, in order */
  uint64_t* drop_bytes;
  int32_t* drop_reason;
  size_t drop_cap, n_drops;
} leveldb_log_replay_out;

/*
 * Replay log::Reader::ReadRecord until it returns false, over the scan
 * (rec_off/rec_len/n_rec from leveldb_log_scan with the same file and
 * initial_offset) and the per-record check results rec_bad[i] (non-zero =
 * stored crc != crc32c(type || payload); ignored, and may be NULL, when
 * checksum == 0).  Capacities: n_rec records and fragments and
 * 2 * (n_rec + size / 32768 + 2) drops always suffice; LEVELDB_LOG_ECAPACITY
 * otherwise.  LEVELDB_LOG_EINVAL if the scan does not match the file.
 */
int leveldb_log_replay(const void* file, size_t size, uint64_t initial_offset, int checksum,
                       const uint64_t* rec_off, const uint32_t* rec_len, const uint8_t* rec_bad,
                       size_t n_rec, leveldb_log_replay_out* out);

/* The Status::Corruption(reason).ToString() text for a drop_reason code, as
 * the reference Reporter receives it ("Corruption: checksum mismatch").
 * Writes at most n bytes including the terminating NUL; returns buf. */
const char* leveldb_log_reason(int32_t code, char* buf, size_t n);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* PRISMDB_LOG_H_ */
