// log_reader.cc -- batched log-record checking, host side (include/prismdb_log.h).
//
// The reference checks log records one at a time inside log::Reader
// (db/log_reader.cc).  Here the checks are hoisted out: leveldb_log_scan lists
// the physical records, the device checks them all in one batch
// (PRISMDB_CRC32C_LOG_HEADER), and leveldb_log_replay re-runs the reader's
// control flow with the batch's answers, so records, LastRecordOffset() values
// and Reporter::Corruption calls come out exactly as the reference produces
// them.  The file is a memory image; reads are the reader's 32 KiB block reads
// (db/log_reader.cc:194-207) and never fail.
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "../../include/prismdb_log.h"

namespace {

constexpr uint64_t kBlock = LEVELDB_LOG_BLOCK_SIZE;
constexpr uint64_t kHeader = LEVELDB_LOG_HEADER_SIZE;

// log_format.h record types, and the reader's two pseudo-types (log_reader.h).
enum : unsigned {
  kZero = 0,
  kFull = 1,
  kFirst = 2,
  kMiddle = 3,
  kLast = 4,
  kEofPseudo = 5,
  kBadPseudo = 6,
};

// Where the reader starts: db/log_reader.cc:34-55 (SkipToInitialBlock).  A
// block start within 6 bytes of the end holds only a trailer and is skipped.
uint64_t FirstBlock(uint64_t initial_offset) {
  const uint64_t in_block = initial_offset % kBlock;
  uint64_t start = initial_offset - in_block;
  if (in_block > kBlock - 6) start += kBlock;
  return start;
}

struct Header {
  uint32_t length;
  unsigned type;  // as the reader sees it: header[6] through a signed char
};

Header ParseHeader(const uint8_t* h) {
  Header r;
  r.length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
  r.type = (unsigned)(int)(signed char)h[6];
  return r;
}

// The reader's buffer as file coordinates: buffer_ == file[pos, end), and
// end_of_buffer_offset_ == end (reads are sequential from the first block).
class Replayer {
 public:
  Replayer(const uint8_t* f, uint64_t size, uint64_t initial_offset, bool checksum,
           const uint64_t* rec_off, const uint32_t* rec_len, const uint8_t* rec_bad, size_t n_rec,
           leveldb_log_replay_out* out)
      : f_(f), size_(size), initial_(initial_offset), checksum_(checksum), rec_off_(rec_off),
        rec_len_(rec_len), rec_bad_(rec_bad), n_rec_(n_rec), out_(out), resyncing_(initial_offset > 0) {}

  int Run() {
    out_->n_records = out_->n_fragments = out_->n_drops = 0;
    // ReadRecord until it returns false (db/log_reader.cc:57-176).
    for (;;) {
      int rc = 0;
      const bool got = ReadRecord(&rc);
      if (rc != 0) return rc;
      if (!got) return 0;
    }
  }

 private:
  // One physical record: db/log_reader.cc:190-273.  Returns its type (or a
  // pseudo-type); *k = its index in the scan when one was returned.
  unsigned ReadPhysical(size_t* k, int* rc) {
    for (;;) {
      if (end_ - pos_ < kHeader) {
        if (!eof_) {  // trailer (or nothing) left: next block
          const uint64_t n = std::min<uint64_t>(kBlock, size_ - end_);
          pos_ = end_;
          end_ += n;
          if (n < kBlock) eof_ = true;
          continue;
        }
        pos_ = end_;  // truncated header at the end of the file: EOF, no report
        return kEofPseudo;
      }
      const Header h = ParseHeader(f_ + pos_);
      if (kHeader + h.length > end_ - pos_) {
        const uint64_t drop = end_ - pos_;
        pos_ = end_;
        if (!eof_) {
          Drop(drop, LEVELDB_LOG_BAD_RECORD_LENGTH);
          return kBadPseudo;
        }
        return kEofPseudo;  // writer died mid-record
      }
      if (h.type == kZero && h.length == 0) {  // preallocated region: skip the block silently
        pos_ = end_;
        return kBadPseudo;
      }
      const uint64_t at = pos_;
      const size_t idx = Find(at);
      if (idx == n_rec_ || rec_len_[idx] != h.length) {
        *rc = LEVELDB_LOG_EINVAL;  // the scan does not describe this file
        return kEofPseudo;
      }
      if (checksum_ && rec_bad_[idx]) {
        const uint64_t drop = end_ - pos_;
        pos_ = end_;  // the length may be the corrupted field: drop the block
        Drop(drop, LEVELDB_LOG_CHECKSUM_MISMATCH);
        return kBadPseudo;
      }
      pos_ += kHeader + h.length;
      *k = idx;
      if (at < initial_) return kBadPseudo;  // started before initial_offset: skipped, no fragment
      return h.type;
    }
  }

  bool ReadRecord(int* rc) {
    if (last_record_offset_ < initial_) {
      // db/log_reader.cc:58-62 (the reader only gets here on its first call)
      const uint64_t start = FirstBlock(initial_);
      if (start > size_) return false;  // Skip() past the end fails: no records
      pos_ = end_ = start;
    }
    bool in_fragmented = false;
    uint64_t scratch_bytes = 0;
    uint32_t scratch_first = (uint32_t)out_->n_fragments;
    uint64_t prospective = 0;
    for (;;) {
      size_t k = (size_t)-1;
      const unsigned type = ReadPhysical(&k, rc);
      if (*rc != 0) return false;
      // Fragment length and header offset: only read for real record types,
      // which always come with their scan index.
      const uint64_t frag_len = k != (size_t)-1 ? rec_len_[k] : 0;
      const uint64_t phys_off = k != (size_t)-1 ? rec_off_[k] : 0;
      if (resyncing_) {  // db/log_reader.cc:79-89
        if (type == kMiddle) continue;
        if (type == kLast) {
          resyncing_ = false;
          continue;
        }
        resyncing_ = false;
      }
      switch (type) {
        case kFull:
          if (in_fragmented && scratch_bytes != 0) Drop(scratch_bytes, LEVELDB_LOG_PARTIAL_NO_END_1);
          out_->n_fragments = scratch_first;  // discard any partial fragments
          if (!PushFragment(k, rc) || !PushRecord(phys_off, scratch_first, 1, rc)) return false;
          last_record_offset_ = phys_off;
          return true;
        case kFirst:
          if (in_fragmented && scratch_bytes != 0) Drop(scratch_bytes, LEVELDB_LOG_PARTIAL_NO_END_2);
          prospective = phys_off;
          out_->n_fragments = scratch_first;
          if (!PushFragment(k, rc)) return false;
          scratch_bytes = frag_len;
          in_fragmented = true;
          break;
        case kMiddle:
          if (!in_fragmented) {
            Drop(frag_len, LEVELDB_LOG_MISSING_START_1);
          } else {
            if (!PushFragment(k, rc)) return false;
            scratch_bytes += frag_len;
          }
          break;
        case kLast:
          if (!in_fragmented) {
            Drop(frag_len, LEVELDB_LOG_MISSING_START_2);
          } else {
            if (!PushFragment(k, rc)) return false;
            if (!PushRecord(prospective, scratch_first, (uint32_t)(out_->n_fragments - scratch_first), rc))
              return false;
            last_record_offset_ = prospective;
            return true;
          }
          break;
        case kEofPseudo:
          out_->n_fragments = scratch_first;
          return false;
        case kBadPseudo:
          if (in_fragmented) {
            Drop(scratch_bytes, LEVELDB_LOG_ERROR_IN_MIDDLE);
            in_fragmented = false;
            scratch_bytes = 0;
            out_->n_fragments = scratch_first;
          }
          break;
        default:
          Drop(frag_len + (in_fragmented ? scratch_bytes : 0),
               LEVELDB_LOG_UNKNOWN_TYPE_BASE + (int32_t)(type & 0xffu));
          in_fragmented = false;
          scratch_bytes = 0;
          out_->n_fragments = scratch_first;
          break;
      }
    }
  }

  // Reporter gate of db/log_reader.cc:183-188 (unsigned arithmetic, as there).
  void Drop(uint64_t bytes, int32_t reason) {
    if (end_ - (end_ - pos_) - bytes < initial_) return;
    if (out_->n_drops < out_->drop_cap) {
      out_->drop_bytes[out_->n_drops] = bytes;
      out_->drop_reason[out_->n_drops] = reason;
    } else {
      overflow_ = true;
    }
    ++out_->n_drops;
  }

  bool PushFragment(size_t k, int* rc) {
    if (out_->n_fragments >= out_->fragment_cap) {
      *rc = LEVELDB_LOG_ECAPACITY;
      return false;
    }
    out_->fragment[out_->n_fragments++] = (uint32_t)k;
    return true;
  }

  bool PushRecord(uint64_t offset, uint32_t first, uint32_t nfrag, int* rc) {
    if (out_->n_records >= out_->record_cap || overflow_) {
      *rc = LEVELDB_LOG_ECAPACITY;
      return false;
    }
    out_->record_offset[out_->n_records] = offset;
    out_->record_first[out_->n_records] = first;
    out_->record_nfrag[out_->n_records] = nfrag;
    ++out_->n_records;
    return true;
  }

  size_t Find(uint64_t at) const {
    const uint64_t* p = std::lower_bound(rec_off_, rec_off_ + n_rec_, at);
    return (p != rec_off_ + n_rec_ && *p == at) ? (size_t)(p - rec_off_) : n_rec_;
  }

  const uint8_t* f_;
  uint64_t size_, initial_;
  bool checksum_;
  const uint64_t* rec_off_;
  const uint32_t* rec_len_;
  const uint8_t* rec_bad_;
  size_t n_rec_;
  leveldb_log_replay_out* out_;
  bool resyncing_;
  bool eof_ = false;
  bool overflow_ = false;
  uint64_t pos_ = 0, end_ = 0;
  uint64_t last_record_offset_ = 0;
};

}  // namespace

extern "C" {

int leveldb_log_scan(const void* file, size_t size, uint64_t initial_offset, uint64_t* rec_off,
                     uint32_t* rec_len, size_t cap, size_t* n_out) {
  if ((file == nullptr && size != 0) || n_out == nullptr || (cap != 0 && (rec_off == nullptr || rec_len == nullptr)))
    return LEVELDB_LOG_EINVAL;
  const uint8_t* f = static_cast<const uint8_t*>(file);
  size_t n = 0;
  // Same walk as the replay, minus the checks: every header a block's chain of
  // length fields reaches, until a trailer, a bad length or a zero record.
  for (uint64_t block = FirstBlock(initial_offset); block < size; block += kBlock) {
    const uint64_t end = std::min<uint64_t>(block + kBlock, size);
    uint64_t pos = block;
    while (end - pos >= kHeader) {
      const Header h = ParseHeader(f + pos);
      if (kHeader + h.length > end - pos) break;
      if (h.type == kZero && h.length == 0) break;
      if (n < cap) {
        rec_off[n] = pos;
        rec_len[n] = h.length;
      }
      ++n;
      pos += kHeader + h.length;
    }
  }
  *n_out = n;
  return n > cap ? LEVELDB_LOG_ECAPACITY : 0;
}

int leveldb_log_replay(const void* file, size_t size, uint64_t initial_offset, int checksum,
                       const uint64_t* rec_off, const uint32_t* rec_len, const uint8_t* rec_bad,
                       size_t n_rec, leveldb_log_replay_out* out) {
  if ((file == nullptr && size != 0) || out == nullptr || (n_rec != 0 && (rec_off == nullptr || rec_len == nullptr)) ||
      (checksum && n_rec != 0 && rec_bad == nullptr))
    return LEVELDB_LOG_EINVAL;
  Replayer r(static_cast<const uint8_t*>(file), size, initial_offset, checksum != 0, rec_off, rec_len, rec_bad,
             n_rec, out);
  const int rc = r.Run();
  if (rc != 0) return rc;
  return out->n_drops > out->drop_cap ? LEVELDB_LOG_ECAPACITY : 0;
}

const char* leveldb_log_reason(int32_t code, char* buf, size_t n) {
  if (buf == nullptr || n == 0) return buf;
  const char* s = nullptr;
  switch (code) {
    case LEVELDB_LOG_CHECKSUM_MISMATCH: s = "checksum mismatch"; break;
    case LEVELDB_LOG_BAD_RECORD_LENGTH: s = "bad record length"; break;
    case LEVELDB_LOG_PARTIAL_NO_END_1: s = "partial record without end(1)"; break;
    case LEVELDB_LOG_PARTIAL_NO_END_2: s = "partial record without end(2)"; break;
    case LEVELDB_LOG_MISSING_START_1: s = "missing start of fragmented record(1)"; break;
    case LEVELDB_LOG_MISSING_START_2: s = "missing start of fragmented record(2)"; break;
    case LEVELDB_LOG_ERROR_IN_MIDDLE: s = "error in middle of record"; break;
    default: break;
  }
  if (s != nullptr) {
    std::snprintf(buf, n, "Corruption: %s", s);
  } else if (code >= LEVELDB_LOG_UNKNOWN_TYPE_BASE && code < LEVELDB_LOG_UNKNOWN_TYPE_BASE + 256) {
    const unsigned type = (unsigned)(int)(signed char)(uint8_t)(code - LEVELDB_LOG_UNKNOWN_TYPE_BASE);
    std::snprintf(buf, n, "Corruption: unknown record type %u", type);
  } else {
    std::snprintf(buf, n, "Corruption: unknown reason %d", (int)code);
  }
  return buf;
}

}  // extern "C"
