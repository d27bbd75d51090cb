/*
 * prismdb_sst.h -- SST layout walker for whole-file batch checksumming
 * (Footer -> index -> BlockHandles -> one verify batch).
 *
 * Reference formats: Footer/BlockHandle table/format.h:23-79 and
 * table/format.cc:17-64; block entries table/block.cc:44-66; filter block
 * discovery table/table.cc (ReadMeta); block trailer table/format.h:79.
 */
#ifndef PRISMDB_SST_H_
#define PRISMDB_SST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRISMDB_SST_ECORRUPT (-10)  /* message: the reference's Status text */
#define PRISMDB_SST_ECAPACITY (-11) /* *n_out holds the count needed */
#define PRISMDB_SST_EUNSUPPORTED (-12) /* "Not implemented: ...": a snappy-compressed
                                          index block */

/* block kinds */
#define PRISMDB_SST_DATA 0
#define PRISMDB_SST_FILTER 1
#define PRISMDB_SST_METAINDEX 2
#define PRISMDB_SST_INDEX 3

/*
 * List the blocks of an SST image in host memory as checksum spans:
 * span i = file[off[i], off[i] + len[i]) = contents || type (len = size + 1),
 * its stored masked CRC in the 4 bytes that follow.  Order: data blocks in
 * index order, filter block (if any), metaindex, index.  The index block's
 * own checksum is verified on the host before it is parsed (a mismatch returns
 * PRISMDB_SST_ECORRUPT, "Corruption: block checksum mismatch"), and its type
 * byte is dispatched as ReadBlock does (table/format.cc:104-146): any type but
 * kNoCompression/kSnappyCompression is "Corruption: bad block type".
 *
 * Limit: the walker does not decompress.  Tables written with
 * Options::compression = kSnappyCompression (table/table_builder.cc:159) may
 * hold a snappy index block; that returns PRISMDB_SST_EUNSUPPORTED instead
 * of a misparse.  A snappy (or any other non-raw type) metaindex is not
 * walked -- no filter span is listed -- but is still listed itself and so
 * verified by the batch; the reference ignores metaindex errors too
 * (Table::ReadMeta, table/table.cc:84-111).  Snappy *data* blocks are
 * fine: their checksum covers the stored (compressed) bytes.  PrismDB's
 * default is kNoCompression (include/leveldb/options.h:134).
 *
 * off/len/kind may be NULL to only count.  Returns 0, PRISMDB_SST_ECORRUPT,
 * PRISMDB_SST_EUNSUPPORTED (reason in leveldb_sst_last_error()) or
 * PRISMDB_SST_ECAPACITY.
 */
int leveldb_sst_block_spans(const char* file, size_t file_size, uint64_t* off, uint32_t* len,
                            uint8_t* kind, size_t cap, size_t* n_out);

const char* leveldb_sst_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* PRISMDB_SST_H_ */
