// oracle/log_fixture.cc -- TEST INFRASTRUCTURE ONLY (fixture generator).
//
// Links the reference log::Writer / log::Reader (db/log_writer.cc,
// db/log_reader.cc, compiled from /root/reference by oracle/Makefile `ref`)
// and records, for a set of log files, what the reference reader returns:
// every logical record (LastRecordOffset, size, crc32c of the bytes) and every
// Reporter::Corruption(bytes, status) call.  The scenarios restate the cases
// of db/log_test.cc (trailers, fragmentation, every corruption path, initial
// offsets) plus seeded random corruptions.  Output (data only):
//   <out>.bin   the log files, back to back
//   <out>.json  one object per case: name, file slice, initial_offset,
//               checksum, records [[offset, size, crc]], drops [[bytes, msg]]
// Nothing here is shipped: tests/ compare prismdb_amd.log against the JSON.
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "db/log_format.h"
#include "db/log_reader.h"
#include "db/log_writer.h"
#include "leveldb/env.h"
#include "leveldb/status.h"
#include "util/coding.h"
#include "util/crc32c.h"
#include "util/random.h"

using leveldb::Slice;
using leveldb::Status;
namespace lg = leveldb::log;

namespace {

struct Sink : leveldb::WritableFile {
  std::string bytes;
  Status Append(const Slice& s) override {
    bytes.append(s.data(), s.size());
    return Status::OK();
  }
  Status Close() override { return Status::OK(); }
  Status Flush() override { return Status::OK(); }
  Status Sync() override { return Status::OK(); }
};

struct Source : leveldb::SequentialFile {
  Slice rest;
  explicit Source(const std::string& f) : rest(f) {}
  Status Read(size_t n, Slice* out, char*) override {
    if (n > rest.size()) n = rest.size();
    *out = Slice(rest.data(), n);
    rest.remove_prefix(n);
    return Status::OK();
  }
  Status Skip(uint64_t n) override {
    if (n > rest.size()) {
      rest = Slice();
      return Status::NotFound("skipped past end");
    }
    rest.remove_prefix(n);
    return Status::OK();
  }
};

struct Drops : lg::Reader::Reporter {
  std::vector<std::pair<size_t, std::string>> v;
  void Corruption(size_t bytes, const Status& s) override { v.emplace_back(bytes, s.ToString()); }
};

struct Case {
  std::string name, file;  // file: the bytes the reader sees
  uint64_t initial_offset;
  bool checksum;
  std::string base;                            // stored file the bytes derive from
  std::vector<std::pair<size_t, int>> edits;   // (position, new byte) applied to base
  size_t keep;                                 // then truncated to keep bytes
};

// A log built by the reference writer, then edited.
struct Log {
  Sink sink;
  lg::Writer* w = new lg::Writer(&sink);
  ~Log() { delete w; }
  Log& add(const std::string& r) {
    w->AddRecord(Slice(r));
    return *this;
  }
  void reopen() {  // log::Writer(dest, dest_length): append to an existing file
    delete w;
    w = new lg::Writer(&sink, sink.bytes.size());
  }
  void fix_checksum(size_t hdr, size_t len) {
    uint32_t c = leveldb::crc32c::Mask(leveldb::crc32c::Value(&sink.bytes[hdr + 6], 1 + len));
    leveldb::EncodeFixed32(&sink.bytes[hdr], c);
  }
};

std::string Repeat(const std::string& s, size_t n) {
  std::string r;
  while (r.size() < n) r += s;
  r.resize(n);
  return r;
}

std::string Num(int i) { return std::to_string(i) + "."; }

std::string JsonStr(const std::string& s) {
  std::string r = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') r += '\\';
    r += c;
  }
  return r + "\"";
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s <out-prefix>\n", argv[0]);
    return 2;
  }
  const size_t B = lg::kBlockSize, H = lg::kHeaderSize;
  std::vector<Case> cases;
  auto push = [&](const std::string& name, const std::string& f, uint64_t init = 0, bool ck = true) {
    cases.push_back(Case{name, f, init, ck, f, {}, f.size()});
  };

  push("empty", "");
  { Log l; l.add("foo").add("bar").add("").add("xxxx"); push("read_write", l.sink.bytes); }
  { Log l; for (int i = 0; i < 5000; ++i) l.add(Num(i)); push("many_blocks", l.sink.bytes); }
  {
    Log l;
    l.add("small").add(Repeat("medium", 50000)).add(Repeat("large", 100000));
    push("fragmentation", l.sink.bytes);
  }
  { Log l; l.add(Repeat("foo", B - 2 * H)).add("").add("bar"); push("marginal_trailer", l.sink.bytes); }
  { Log l; l.add(Repeat("foo", B - 2 * H)).add("bar"); push("marginal_trailer2", l.sink.bytes); }
  { Log l; l.add(Repeat("foo", B - 2 * H + 4)).add("").add("bar"); push("short_trailer", l.sink.bytes); }
  { Log l; l.add(Repeat("foo", B - 2 * H + 4)); push("aligned_eof", l.sink.bytes); }
  { Log l; l.add("hello"); l.reopen(); l.add("world"); push("open_for_append", l.sink.bytes); }
  {
    Log l;
    leveldb::Random rnd(301);
    for (int i = 0; i < 500; ++i) l.add(Repeat(Num(i), rnd.Skewed(14)));
    push("random_read", l.sink.bytes);
  }
  { Log l; l.add("foo"); l.sink.bytes[6] += 100; l.fix_checksum(0, 3); push("bad_record_type", l.sink.bytes); }
  { Log l; l.add("foo"); l.sink.bytes.resize(l.sink.bytes.size() - 4); push("truncated_trailing", l.sink.bytes); }
  { Log l; l.add(Repeat("bar", B - H)).add("foo"); l.sink.bytes[4] += 1; push("bad_length", l.sink.bytes); }
  { Log l; l.add("foo"); l.sink.bytes.resize(l.sink.bytes.size() - 1); push("bad_length_at_end", l.sink.bytes); }
  {
    Log l;
    l.add("foo");
    l.sink.bytes[0] += 10;
    push("checksum_mismatch", l.sink.bytes);
    push("checksum_mismatch_unchecked", l.sink.bytes, 0, false);
  }
  { Log l; l.add("foo"); l.sink.bytes[6] = lg::kMiddleType; l.fix_checksum(0, 3); push("unexpected_middle", l.sink.bytes); }
  { Log l; l.add("foo"); l.sink.bytes[6] = lg::kLastType; l.fix_checksum(0, 3); push("unexpected_last", l.sink.bytes); }
  {
    Log l;
    l.add("foo").add("bar");
    l.sink.bytes[6] = lg::kFirstType;
    l.fix_checksum(0, 3);
    push("unexpected_full", l.sink.bytes);
  }
  {
    Log l;
    l.add("foo").add(Repeat("bar", 100000));
    l.sink.bytes[6] = lg::kFirstType;
    l.fix_checksum(0, 3);
    push("unexpected_first", l.sink.bytes);
  }
  { Log l; l.add(Repeat("bar", B)); l.sink.bytes.resize(l.sink.bytes.size() - 14); push("missing_last", l.sink.bytes); }
  { Log l; l.add(Repeat("bar", B)); l.sink.bytes.resize(l.sink.bytes.size() - 1); push("partial_last", l.sink.bytes); }
  { Log l; l.add(Repeat("foo", 3 * B)).add("correct"); push("skip_into_multi_record", l.sink.bytes, B); }
  {
    Log l;
    l.add(Repeat("foo", B)).add(Repeat("bar", B)).add("correct");
    for (size_t o = B; o < 2 * B; ++o) l.sink.bytes[o] = 'x';
    push("error_joins_records", l.sink.bytes);
    push("error_joins_records_unchecked", l.sink.bytes, 0, false);
  }
  {
    // db/log_test.cc's initial-offset log: six records, the third spans three
    // blocks, the fifth leaves a 2-byte block trailer, the sixth fills block 4.
    Log l;
    const size_t sizes[] = {10000, 10000, 2 * B - 1000, 1, 13716, B - H};
    for (int i = 0; i < 6; ++i) l.add(std::string(sizes[i], (char)('a' + i)));
    const std::string f = l.sink.bytes;
    const uint64_t offs[] = {0, 1, 10000, 10007, 10008, 20014, 20015, B - 4, B + 1, 2 * B + 1,
                             2 * (H + 10000) + (2 * B - 1000) + 3 * H, 3 * B - 3, 3 * B, f.size(),
                             f.size() + 5, f.size() + B};
    for (uint64_t o : offs) push("initial_offset_" + std::to_string(o), f, o);
  }
  {
    // preallocated (zero) regions: type 0 / length 0 headers
    Log l;
    l.add("alpha").add(Repeat("beta", 40000));
    std::string f = l.sink.bytes + std::string(3000, '\0');
    push("zero_tail", f);
    Log m;
    m.add("one");
    std::string g = m.sink.bytes + std::string(B - m.sink.bytes.size(), '\0');
    Log k;
    k.add("two").add(Repeat("three", 70000));
    push("zero_block_then_records", g + k.sink.bytes);
  }
  {
    // seeded random damage on a mixed-size log
    Log base;
    leveldb::Random rnd(7);
    for (int i = 0; i < 400; ++i) base.add(Repeat(Num(i), rnd.Skewed(13)));
    const std::string f = base.sink.bytes;
    std::mt19937_64 g(0x5EED0007);
    for (int c = 0; c < 64; ++c) {
      Case k{"fuzz_" + std::to_string(c), f, 0, c % 8 != 7, f, {}, f.size()};
      const int edits = 1 + (int)(g() % 4);
      for (int e = 0; e < edits; ++e) {
        const size_t pos = g() % f.size();
        int v;
        switch (g() % 3) {
          case 0: v = (uint8_t)k.file[pos] ^ (1 << (g() % 8)); break;
          case 1: v = (int)(g() & 0xff); break;
          default: v = 0; break;
        }
        k.file[pos] = (char)v;
        k.edits.emplace_back(pos, v);
      }
      if (c % 6 == 5) k.keep = f.size() - (g() % 5000);
      k.file.resize(k.keep);
      k.initial_offset = (c % 4 == 3) ? g() % k.keep : 0;
      cases.push_back(k);
    }
  }

  const std::string prefix = argv[1];
  std::ofstream bin(prefix + ".bin", std::ios::binary);
  std::ofstream js(prefix + ".json");
  js << "{\"block_size\": " << B << ", \"header_size\": " << H << ", \"cases\": [\n";
  std::vector<std::pair<std::string, size_t>> stored;  // each distinct base once
  size_t at = 0;
  for (size_t ci = 0; ci < cases.size(); ++ci) {
    const Case& c = cases[ci];
    size_t where = at;
    bool found = false;
    for (const auto& sb : stored)
      if (sb.first == c.base) {
        where = sb.second;
        found = true;
        break;
      }
    if (!found) {
      bin.write(c.base.data(), c.base.size());
      stored.emplace_back(c.base, at);
      at += c.base.size();
    }
    Source src(c.file);
    Drops rep;
    lg::Reader r(&src, &rep, c.checksum, c.initial_offset);
    std::string scratch;
    Slice rec;
    js << " {\"name\": " << JsonStr(c.name) << ", \"offset\": " << where << ", \"size\": " << c.base.size()
       << ", \"keep\": " << c.keep << ", \"edits\": [";
    for (size_t i = 0; i < c.edits.size(); ++i)
      js << (i ? ", " : "") << "[" << c.edits[i].first << ", " << c.edits[i].second << "]";
    js << "], \"initial_offset\": " << c.initial_offset << ", \"checksum\": " << (c.checksum ? "true" : "false")
       << ",\n  \"records\": [";
    int nrec = 0;
    while (r.ReadRecord(&rec, &scratch)) {
      js << (nrec++ ? ", " : "") << "[" << r.LastRecordOffset() << ", " << rec.size() << ", "
         << leveldb::crc32c::Value(rec.data(), rec.size()) << "]";
    }
    js << "],\n  \"drops\": [";
    for (size_t i = 0; i < rep.v.size(); ++i)
      js << (i ? ", " : "") << "[" << rep.v[i].first << ", " << JsonStr(rep.v[i].second) << "]";
    js << "]}" << (ci + 1 < cases.size() ? "," : "") << "\n";
  }
  js << "]}\n";
  std::fprintf(stdout, "%zu cases, %zu bytes\n", cases.size(), at);
  return 0;
}
