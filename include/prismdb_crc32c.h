/*
 * prismdb_crc32c.h -- C ABI of the MI355X batched CRC32C engine.
 *
 * Drop-in boundary for LevelDB/PrismDB's block-checksum path.  Plain C types
 * only (no HIP, no torch): device pointers are `const void*`, the stream is an
 * opaque `void*` (a hipStream_t; NULL = the null stream).  Naming follows the
 * reference's C API (include/leveldb/c.h: `leveldb_` prefix).
 *
 * Reference interfaces each entry point replaces or feeds:
 *   leveldb_crc32c_extend/value   crc32c::Extend / Value          util/crc32c.h:17-20, util/crc32c.cc:276-377
 *   leveldb_crc32c_mask/unmask    crc32c::Mask / Unmask           util/crc32c.h:27-38
 *   leveldb_crc32c_batch*         N x crc32c::Value (+Extend type byte, +Mask) as issued by
 *                                 TableBuilder::WriteRawBlock      table/table_builder.cc:185-202
 *   ..._batch* with mismatch out  N x ReadBlock's verify          table/format.cc:91-102
 *   ..._batch* with LOG_HEADER    N x log::Writer::EmitPhysicalRecord's crc / log::Reader's
 *                                 check                           db/log_writer.cc:94-97, db/log_reader.cc:231-245
 *   leveldb_crc32c_accelerated    crc32c's CanAccelerateCRC32C    util/crc32c.cc:267-274
 *                                 (port::AcceleratedCRC32C hook   port/port_stdcxx.h:141-151)
 *
 * Return convention: 0 = ok, < 0 = error (PRISMDB_CRC32C_E*); the message is in
 * leveldb_crc32c_last_error() (thread-local).  A checksum MISMATCH is data, not
 * an error: callers map mismatch[i] != 0 to Status::Corruption("block checksum
 * mismatch") exactly as table/format.cc:99 does.
 *
 * Threading: every entry point is reentrant; concurrent calls on distinct
 * streams take no lock after the one-time per-device initialisation.
 * Ownership: the caller owns every buffer until the stream work completes; the
 * engine keeps no pointer past the call.
 */
#ifndef PRISMDB_CRC32C_H_
#define PRISMDB_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* flags */
#define PRISMDB_CRC32C_MASK 0x1u /* out[i] = crc32c::Mask(crc)  (table/table_builder.cc:196) */
/* also store the (masked, with MASK) result as 4 LE bytes right after each span,
 * i.e. seal `contents || type` spans with their trailer in place, as
 * TableBuilder::WriteRawBlock does (table/table_builder.cc:192-197).  The
 * buffer must be writable; not combinable with verify (mismatch != NULL). */
#define PRISMDB_CRC32C_WRITE_TRAILER 0x2u
/* log (WAL / MANIFEST) physical-record layout: the stored checksum that verify
 * compares against, and that WRITE_TRAILER writes, is the 4 LE bytes 6 bytes
 * BEFORE the span instead of right after it.  A log record is
 * crc[4] | length[2] | type[1] | payload: pass span = type||payload, i.e.
 * off = record + 6, len = 1 + length (db/log_writer.cc:94-97 computes
 * Mask(Extend(type_crc[t], payload)) == Mask(Value(type||payload));
 * db/log_reader.cc:231-245 checks Value(header + 6, 1 + length)). */
#define PRISMDB_CRC32C_LOG_HEADER 0x4u
/* Accepted and ignored by leveldb_crc32c_batch, batch_fixed and batch_multi
 * (batch_host rejects it); kept so that callers built against round 3's
 * header still link and run.  Every batch runs in stream order: the
 * any-order launch it used to request is not supported on gfx9
 * (hip/hip_ext.h, hipExtAnyOrderLaunch) and measured slower where it ran. */
#define PRISMDB_CRC32C_UNORDERED 0x8u

/* error codes */
#define PRISMDB_CRC32C_EINVAL (-1)  /* bad argument */
#define PRISMDB_CRC32C_EDEVICE (-2) /* HIP runtime error */
#define PRISMDB_CRC32C_ESELFTEST (-3) /* device known-answer self-test failed */

/* ---- per-call host surface (CPU; per-call GPU launches would lose) ---- */

/* crc32c::Extend (util/crc32c.cc:276): crc32c of A||data[0,n) given init_crc = crc32c(A). */
uint32_t leveldb_crc32c_extend(uint32_t init_crc, const char* data, size_t n);
/* crc32c::Value (util/crc32c.h:20) */
uint32_t leveldb_crc32c_value(const char* data, size_t n);
/* crc32c::Mask / Unmask (util/crc32c.h:27-38) */
uint32_t leveldb_crc32c_mask(uint32_t crc);
uint32_t leveldb_crc32c_unmask(uint32_t masked_crc);
/* crc32c of A||B from crc32c(A), crc32c(B), |B| (no reference equivalent; used to stitch split spans). */
uint32_t leveldb_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
/* 1 if the host Extend uses the CPU's CRC32 instruction (KAT-gated like util/crc32c.cc:267-274). */
int leveldb_crc32c_accelerated(void);

/* ---- device batch surface (MI355X) ---- */

/* One-time per-device setup (tables to HBM, device self-test against the
 * util/crc32c.cc:269-273 vector).  Called implicitly by the batch functions;
 * call it explicitly before stream capture. */
int leveldb_crc32c_device_init(int device);

/*
 * Fixed-stride batch: block i = base[i*stride, i*stride + len), i < nblocks.
 *   out[i]      = Extend(init, block_i)         (Mask()ed when flags & MASK)   -- may be NULL
 *   mismatch[i] = Value(block_i) != Unmask(LE32(block_i + len))  (ReadBlock
 *                 verify with len = n+1: contents||type, table/format.cc:93-95) -- may be NULL
 * All pointers are device pointers on the current HIP device.
 */
int leveldb_crc32c_batch_fixed(const void* dev_base, size_t stride, size_t len, size_t nblocks,
                               uint32_t init, uint32_t* dev_out, uint8_t* dev_mismatch,
                               uint32_t flags, void* stream);

/*
 * Variable batch: block i = base[off[i], off[i] + len[i]); init[i] per block
 * (dev_init may be NULL: all 0).  Any byte alignment, any length (< 4 GiB).
 * Long spans are split across many wavefronts and recombined on the device.
 * Routing: <= 2^17 spans one kernel launch (an SST file, a log file);
 * batches that seal (WRITE_TRAILER) or verify block trailers (dev_mismatch
 * != NULL), without LOG_HEADER: one launch up to 196 608 spans (11 SST files
 * of 64 MiB, on a 256-CU device) and two such launches up to 2^18 (a
 * compaction's dozen SST files: uniform blocks run faster that way);
 * everything else the planner path (task-balanced slices: plain checksum
 * batches of mixed span sizes, log records, any batch beyond 2^18 spans).
 */
int leveldb_crc32c_batch(const void* dev_base, const uint64_t* dev_off, const uint32_t* dev_len,
                         const uint32_t* dev_init, size_t n, uint32_t* dev_out,
                         uint8_t* dev_mismatch, uint32_t flags, void* stream);

/*
 * Host-resident batch (blocks still in host memory, e.g. SST pages read by
 * pread during compaction): span i = host_base[off[i], off[i] + len[i]),
 * offsets sorted ascending, each span (+ its 4-byte trailer when verifying)
 * at most 64 MiB.  Streams 64 MiB chunks host -> device (through pinned
 * staging when host_base is pageable; directly when it is pinned/registered)
 * -> batch kernel -> results back, four chunks in flight on the engine's own
 * streams.  Synchronous; out/mismatch are host arrays (either may be NULL).
 * flags: PRISMDB_CRC32C_MASK, PRISMDB_CRC32C_LOG_HEADER (verify log records:
 * the 6 header bytes before each span travel with it), and
 * PRISMDB_CRC32C_WRITE_TRAILER (not with mismatch): each span's (masked)
 * result is stored into host_base as its trailer -- 4 LE bytes right after
 * the span, or with LOG_HEADER the header crc 6 bytes before it -- as
 * TableBuilder::WriteRawBlock appends it (table/table_builder.cc:192-197); the
 * buffer must then be writable and no trailer may overlap a span of the batch.
 * The `const` of host_base does not hold under WRITE_TRAILER (nor does that of
 * dev_base in the device calls): the first and last trailer slots are probed
 * first, and a buffer not writable there (a PROT_READ mapping) is refused with
 * PRISMDB_CRC32C_EINVAL before anything is stored.
 * On an error return, the trailers of chunks already finished may be written.
 * Uses the current HIP device.
 */
int leveldb_crc32c_batch_host(const void* host_base, const uint64_t* off, const uint32_t* len,
                              const uint32_t* init, size_t n, uint32_t* out, uint8_t* mismatch,
                              uint32_t flags);

/*
 * Several devices from one process: PrismDB's partitions (db/db_impl.h:359,
 * one background thread each, util/env_posix.cc:850-890) with partition p's
 * blocks resident on device devices[p].  Each device checksums its batch
 * (span i of partition p = dev_base[p][dev_off[p][i], + dev_len[p][i]),
 * dev_init may be NULL, dev_init[p] may be NULL), then one RCCL gather over
 * xGMI (grouped ncclSend/ncclRecv, communicators from ncclCommInitAll, kept
 * per device list) brings the results to devices[0]: out0 / mismatch0 are
 * device arrays on devices[0] of n[0] + ... + n[ndev-1] entries, partition
 * after partition (either may be NULL, not both).  flags as for
 * leveldb_crc32c_batch (WRITE_TRAILER seals in place on every device).
 * streams may be NULL (null streams) or hold one stream per device: the work
 * is ordered after what is already on streams[p] and streams[p] waits for
 * it.  Calls with the same device list are serialized.
 */
int leveldb_crc32c_batch_multi(int ndev, const int* devices, const void* const* dev_base,
                               const uint64_t* const* dev_off, const uint32_t* const* dev_len,
                               const uint32_t* const* dev_init, const size_t* n, uint32_t* out0,
                               uint8_t* mismatch0, uint32_t flags, void* const* streams);

/* Thread-local message for the last non-zero return on this thread. */
const char* leveldb_crc32c_last_error(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* PRISMDB_CRC32C_H_ */
