// sst_fixture.cc -- TEST INFRASTRUCTURE ONLY (fixture generator: not part of
// the product library; the built binary travels to the GPU box with the tree,
// where tests/test_gpu_sst_full.py runs it to write a full-size reference table).
//
// Drives the reference TableBuilder (table/table_builder.cc, compiled from
// /root/reference by oracle/Makefile) to write a small SST shaped like
// PrismDB's YCSB data (8-byte keys, 980-byte values, block_size 4 KiB,
// kNoCompression -- include/leveldb/options.h:101,134), then re-opens it with
// the reference Table::Open + ReadBlock(verify_checksums) to prove the file is
// clean. Every WriteRawBlock (table/table_builder.cc:185-202) issues exactly
// two Appends: the contents, then the 5-byte trailer; the file sink records
// those so the fixture lists each block's handle and stored trailer.
//
// usage: sst_fixture <out.ldb> <out.json> <nkeys> <value_len> <block_size>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "leveldb/env.h"
#include "leveldb/iterator.h"
#include "leveldb/options.h"
#include "leveldb/table.h"
#include "leveldb/table_builder.h"

namespace {

class RecordingSink : public leveldb::WritableFile {
 public:
  std::string contents;
  std::vector<std::pair<size_t, size_t>> appends;  // (offset, size)
  leveldb::Status Append(const leveldb::Slice& d) override {
    appends.emplace_back(contents.size(), d.size());
    contents.append(d.data(), d.size());
    return leveldb::Status::OK();
  }
  leveldb::Status Close() override { return leveldb::Status::OK(); }
  leveldb::Status Flush() override { return leveldb::Status::OK(); }
  leveldb::Status Sync() override { return leveldb::Status::OK(); }
};

class StringSource : public leveldb::RandomAccessFile {
 public:
  explicit StringSource(const std::string& s) : s_(s) {}
  leveldb::Status Read(uint64_t offset, size_t n, leveldb::Slice* result,
                       char* scratch) const override {
    if (offset >= s_.size()) return leveldb::Status::InvalidArgument("off");
    if (offset + n > s_.size()) n = s_.size() - offset;
    std::memcpy(scratch, s_.data() + offset, n);
    *result = leveldb::Slice(scratch, n);
    return leveldb::Status::OK();
  }

 private:
  std::string s_;
};

uint64_t Mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 6) {
    std::fprintf(stderr, "usage: %s out.ldb out.json nkeys value_len block_size\n", argv[0]);
    return 2;
  }
  const int nkeys = std::atoi(argv[3]);
  const int vlen = std::atoi(argv[4]);
  leveldb::Options opt;
  opt.block_size = (size_t)std::atoi(argv[5]);
  opt.compression = leveldb::kNoCompression;
  opt.paranoid_checks = true;

  RecordingSink sink;
  leveldb::TableBuilder tb(opt, &sink);
  std::string value(vlen, '\0');
  for (int i = 0; i < nkeys; ++i) {
    char key[8];
    uint64_t k = (uint64_t)i * 7919u + 17u;  // 8-byte big-endian keys sort numerically
    for (int b = 0; b < 8; ++b) key[b] = (char)(k >> (56 - 8 * b));
    for (int j = 0; j < vlen; ++j) value[j] = (char)(Mix((uint64_t)i * 4096u + j) & 0xff);
    tb.Add(leveldb::Slice(key, 8), value);
  }
  leveldb::Status s = tb.Finish();
  if (!s.ok()) {
    std::fprintf(stderr, "Finish: %s\n", s.ToString().c_str());
    return 1;
  }

  // Re-open and read every block with verification on (table/format.cc:91-102).
  StringSource src(sink.contents);
  leveldb::Table* table = nullptr;
  s = leveldb::Table::Open(opt, &src, sink.contents.size(), &table);
  if (!s.ok()) {
    std::fprintf(stderr, "Open: %s\n", s.ToString().c_str());
    return 1;
  }
  leveldb::ReadOptions ro;
  ro.verify_checksums = true;
  leveldb::Iterator* it = table->NewIterator(ro);
  int seen = 0;
  for (it->SeekToFirst(); it->Valid(); it->Next()) ++seen;
  if (!it->status().ok() || seen != nkeys) {
    std::fprintf(stderr, "verify failed: %s seen=%d\n", it->status().ToString().c_str(), seen);
    return 1;
  }
  delete it;
  delete table;

  FILE* f = std::fopen(argv[1], "wb");
  std::fwrite(sink.contents.data(), 1, sink.contents.size(), f);
  std::fclose(f);

  // appends = [contents, trailer]* footer
  const size_t na = sink.appends.size();
  FILE* j = std::fopen(argv[2], "w");
  std::fprintf(j, "{\n  \"generator\": \"oracle/sst_fixture.cc via reference TableBuilder\",\n");
  std::fprintf(j, "  \"nkeys\": %d, \"value_len\": %d, \"block_size\": %zu,\n", nkeys, vlen,
               opt.block_size);
  std::fprintf(j, "  \"file_size\": %zu,\n  \"blocks\": [\n", sink.contents.size());
  for (size_t a = 0; a + 1 < na; a += 2) {
    size_t off = sink.appends[a].first, n = sink.appends[a].second;
    const unsigned char* t = (const unsigned char*)sink.contents.data() + off + n;
    unsigned masked = t[1] | (t[2] << 8) | (t[3] << 16) | ((unsigned)t[4] << 24);
    const char* kind = (a + 3 == na) ? "index" : (a + 5 == na) ? "metaindex" : "data";
    std::fprintf(j, "    {\"offset\": %zu, \"size\": %zu, \"type\": %u, \"masked_crc\": %u, \"kind\": \"%s\"}%s\n",
                 off, n, (unsigned)t[0], masked, kind, (a + 3 < na) ? "," : "");
  }
  std::fprintf(j, "  ],\n  \"footer_offset\": %zu\n}\n", sink.appends[na - 1].first);
  std::fclose(j);
  std::printf("wrote %zu bytes, %zu blocks, verified %d keys\n", sink.contents.size(), (na - 1) / 2,
              seen);
  return 0;
}
