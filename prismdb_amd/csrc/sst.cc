// sst.cc -- SST layout walker for whole-file batch checksumming.
//
// Lists every block of a LevelDB table image the way Table::Open + the
// iterators would ReadBlock them: Footer (last 48 bytes, table/format.h:48-76,
// codecs table/format.cc:17-64) -> index block (entries of table/block.cc:44-66
// whose values are BlockHandles) -> data blocks; metaindex block -> filter
// block ("filter.<policy>", table/table.cc ReadMeta); plus the metaindex and
// index blocks themselves.  Each block becomes one span `contents || type`
// (size + 1 bytes) whose stored trailer follows it -- exactly what
// ReadBlock's verify covers (table/format.cc:91-102).
//
// The index block is parsed before the device batch runs, so its own trailer
// is checked first on the host (one block, the per-call Extend), as
// Table::Open does for paranoid reads (table/table.cc:60-66).
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/prismdb_crc32c.h"
#include "../../include/prismdb_sst.h"
#include "../../include/util/crc32c.h"

namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;  // table/format.h:76
constexpr size_t kFooterLen = 48;                         // 2 * 20 + 8, table/format.h:54
constexpr size_t kTrailerLen = 5;                         // table/format.h:79

thread_local std::string t_sst_error;

inline uint32_t Le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Little-endian base-128 varints (util/coding.cc:86-131): at most 5 / 10 bytes.
bool ReadVarint(const uint8_t*& p, const uint8_t* end, int max_bytes, uint64_t* v) {
  uint64_t r = 0;
  for (int i = 0, shift = 0; i < max_bytes && p < end; ++i, shift += 7) {
    const uint64_t b = *p++;
    r |= (b & 0x7f) << shift;
    if ((b & 0x80) == 0) {
      *v = r;
      return true;
    }
  }
  return false;
}

struct Handle {
  uint64_t offset = 0, size = 0;
};

bool ReadHandle(const uint8_t*& p, const uint8_t* end, Handle* h) {
  return ReadVarint(p, end, 10, &h->offset) && ReadVarint(p, end, 10, &h->size);
}

int Corrupt(const std::string& why) {
  t_sst_error = "Corruption: " + why;
  return PRISMDB_SST_ECORRUPT;
}

// Status::NotSupported's text (util/status.cc: "Not implemented: ").
int Unsupported(const std::string& what) {
  t_sst_error = "Not implemented: " + what;
  return PRISMDB_SST_EUNSUPPORTED;
}

// Block types, table/format.h (CompressionType, include/leveldb/options.h:25-31).
constexpr uint8_t kNoCompression = 0;
constexpr uint8_t kSnappyCompression = 1;

// ReadBlock's verify for one block on the host: contents || type against the
// stored masked CRC that follows (table/format.cc:93-101).
bool HostVerify(const uint8_t* block, uint64_t size) {
  return leveldb::crc32c::Unmask(Le32(block + size + 1)) ==
         leveldb::crc32c::Value(reinterpret_cast<const char*>(block), (size_t)size + 1);
}

struct Table {
  const uint8_t* file;
  size_t size;
  // A block (contents plus 5-byte trailer) must fit before the footer.
  bool Fits(const Handle& h) const {
    return h.offset <= size && h.size <= size && h.offset + h.size + kTrailerLen <= size - kFooterLen;
  }
};

// Visit the entries of a block (table/block.cc layout: entries with
// prefix-compressed keys, then uint32 restarts[num], then uint32 num).  The
// callback gets the full key and the value.
template <typename Fn>
bool ForEachEntry(const uint8_t* data, size_t n, Fn&& fn) {
  if (n < 4) return false;
  const uint32_t num_restarts = Le32(data + n - 4);
  if (num_restarts > (n - 4) / 4) return false;
  const uint8_t* p = data;
  const uint8_t* limit = data + n - 4 * (1 + (size_t)num_restarts);
  std::string key;
  while (p < limit) {
    uint64_t shared, non_shared, vlen;
    if (!ReadVarint(p, limit, 5, &shared) || !ReadVarint(p, limit, 5, &non_shared) ||
        !ReadVarint(p, limit, 5, &vlen))
      return false;
    if ((uint64_t)(limit - p) < non_shared + vlen || shared > key.size()) return false;
    key.resize((size_t)shared);
    key.append(reinterpret_cast<const char*>(p), (size_t)non_shared);
    p += non_shared;
    if (!fn(key, p, (size_t)vlen)) return false;
    p += vlen;
  }
  return true;
}

}  // namespace

extern "C" {

int leveldb_sst_block_spans(const char* file, size_t file_size, uint64_t* off, uint32_t* len,
                            uint8_t* kind, size_t cap, size_t* n_out) {
  *n_out = 0;
  if (file == nullptr && file_size != 0) return Corrupt("null file image");
  const uint8_t* f = reinterpret_cast<const uint8_t*>(file);
  if (file_size < kFooterLen) return Corrupt("file is too short to be an sstable");
  const uint8_t* foot = f + file_size - kFooterLen;
  const uint64_t magic = (uint64_t)Le32(foot + kFooterLen - 8) | ((uint64_t)Le32(foot + kFooterLen - 4) << 32);
  if (magic != kTableMagic) return Corrupt("not an sstable (bad magic number)");
  Handle meta, index;
  const uint8_t* p = foot;
  if (!ReadHandle(p, foot + kFooterLen - 8, &meta) || !ReadHandle(p, foot + kFooterLen - 8, &index))
    return Corrupt("bad block handle");
  const Table t{f, file_size};
  if (!t.Fits(index) || !t.Fits(meta)) return Corrupt("truncated block read");

  // The index is parsed here, so verify it first (ReadBlock, table/format.cc:93-101),
  // then dispatch on its type byte as ReadBlock does (:104-146).  Snappy
  // blocks (Options::compression = kSnappyCompression, table_builder.cc:159)
  // would need decompression before parsing, which this walker does not do.
  const uint8_t* ib = f + index.offset;
  if (!HostVerify(ib, index.size)) return Corrupt("block checksum mismatch");
  if (ib[index.size] == kSnappyCompression) return Unsupported("snappy-compressed index block");
  if (ib[index.size] != kNoCompression) return Corrupt("bad block type");

  std::vector<Handle> spans;
  std::vector<uint8_t> kinds;
  bool ok = ForEachEntry(ib, (size_t)index.size, [&](const std::string&, const uint8_t* v, size_t vn) {
    Handle h;
    const uint8_t* q = v;
    if (!ReadHandle(q, v + vn, &h) || !t.Fits(h)) return false;
    spans.push_back(h);
    kinds.push_back(PRISMDB_SST_DATA);
    return true;
  });
  if (!ok) return Corrupt("bad block contents (index)");

  // Metaindex: "filter.<name>" -> filter block.  Its own trailer is part of
  // the batch, so a damaged metaindex shows up as a mismatch; it is only
  // walked if it is stored uncompressed and parses.  A snappy or unknown-type
  // metaindex is not walked (no filter span) but still verified: the
  // reference does not propagate metaindex errors either (Table::ReadMeta,
  // table/table.cc:84-111, "Do not propagate errors"), Table::Open succeeds.
  const uint8_t* mb = f + meta.offset;
  if (mb[meta.size] == kNoCompression)
    ForEachEntry(mb, (size_t)meta.size, [&](const std::string& key, const uint8_t* v, size_t vn) {
      if (key.compare(0, 7, "filter.") == 0) {
        Handle h;
        const uint8_t* q = v;
        if (ReadHandle(q, v + vn, &h) && t.Fits(h)) {
          spans.push_back(h);
          kinds.push_back(PRISMDB_SST_FILTER);
        }
      }
      return true;
    });
  spans.push_back(meta);
  kinds.push_back(PRISMDB_SST_METAINDEX);
  spans.push_back(index);
  kinds.push_back(PRISMDB_SST_INDEX);

  *n_out = spans.size();
  if (spans.size() > cap) {
    t_sst_error = "capacity too small";
    return PRISMDB_SST_ECAPACITY;
  }
  for (size_t i = 0; i < spans.size(); ++i) {
    if (spans[i].size + 1 > 0xFFFFFFFFull) return Corrupt("block larger than 4 GiB");
    if (off) off[i] = spans[i].offset;
    if (len) len[i] = (uint32_t)(spans[i].size + 1);  // contents || type
    if (kind) kind[i] = kinds[i];
  }
  return 0;
}

const char* leveldb_sst_last_error(void) { return t_sst_error.c_str(); }

}  // extern "C"
