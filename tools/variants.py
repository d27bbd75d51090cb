#!/usr/bin/env python3
"""Compare variants of the engine in ONE process, interleaved.

    python tools/variants.py build [--only a b]     # here: build tools/vlib/lib_*.so
    python tools/variants.py run [--gib 64] ...     # GPU box: time them on one buffer

A variant is the full library built from a PATCHED COPY of the sources
(build/variants/<name>/pkg/csrc; the libraries go to tools/vlib/, which
ships to the GPU box: `build` empties it first, so only the variants built
last travel): each entry of VARIANTS lists exact
text substitutions (file, old, new), each of which must match exactly once.
Measurement-only variants (marked "wrong results") exist only here, never as
knobs in the product source.  Each library is loaded with RTLD_LOCAL and
driven through its own C ABI on the same device buffer; results are compared
across variants (`agree`).  Libraries built elsewhere (e.g. from an older
commit in a git worktree) and dropped into VDIR as lib_<name>.so join the
comparison with --only <name>.

Earlier rounds' -D knob variants (profiles/r01_variants_*, r02*_variants_*)
were measured with the knobs then in the source; those knobs are gone.
"""
import argparse
import ctypes
import json
import os
import shutil
import statistics
import subprocess
import sys

os.environ.setdefault("PRISMDB_ENABLE_TEST_HOOKS", "1")  # the library's prismdb_* setters act only with this
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.environ.get("PRISMDB_VLIB", os.path.join(ROOT, "tools", "vlib"))  # (override: trial builds)

# Measurement-only variants compute wrong results on purpose: their device
# self-test would refuse the device, so it is reported but not enforced.
MEASURE_ONLY = [("crc32c_capi.hip", "  ctx.status = SelfTest(ctx);\n", "  (void)SelfTest(ctx);\n")]

# name -> [(file under prismdb_amd/csrc, old text, new text), ...]
VARIANTS = {
    "base": [],
    # an identical copy under another name: A/A check of the harness
    "base2": [],
    # twice the ticket workers (nwaves / 16)
    "workers2x": [("crc32c_direct.hip", "  uint32_t reserve = nwaves / 32u;", "  uint32_t reserve = nwaves / 16u;")],
    # measurement-only (wrong results: no header written): the lane kernel
    # sealing without its scattered header-crc stores -- what they cost
    "lane_noseal": [("crc32c_kernels.hip",
                     '          asm volatile("global_store_dword %0, %1, off" : : "v"(ta), "v"(v) : "memory");\n',
                     '          (void)ta;\n')] + MEASURE_ONLY,
    # the sealing lane kernel's side load of a record's last task reads the
    # dword holding its header crc (unused: HD is only read at task 0), so
    # that the line is in L2 when the crc is stored
    "lane_seal_touch": [("crc32c_kernels.hip",
                         "    if (kSideAlways || t.k == 0) HD[sl] = asm_load_u32(owned && t.k == 0 ? vp & ~3ull : zero);\n",
                         "    if (kSideAlways || t.k == 0)\n"
                         "      HD[sl] = asm_load_u32(owned && t.k == 0 ? vp & ~3ull\n"
                         "                            : (!kVerify && owned && lastk && (a.flags & kFlagWriteTrailer))\n"
                         "                                  ? (hdr ? vp - kLogCrcBack : vp + vlen) & ~3ull : zero);\n")],
    # span / fixed kernels at 12 and 8 waves per CU (768- / 512-thread groups)
    "waves12": [("crc32c_device.h", "constexpr int kWavesPerGroup = 16;", "constexpr int kWavesPerGroup = 12;")],
    "waves8": [("crc32c_device.h", "constexpr int kWavesPerGroup = 16;", "constexpr int kWavesPerGroup = 8;")],
    # the one-launch kernel's ticket sizing without the batch-size term (<= 64 tickets per span)
    "tlg64": [("crc32c_direct.hip",
               "  const int32_t l = (int32_t)(31u - (uint32_t)__builtin_clz(2u * nwaves)) - (int32_t)ceil_lg(n);\n"
               "  const uint32_t lt = l < 6 ? 6u : (l > 12 ? 12u : (uint32_t)l);\n",
               "  (void)n;\n  (void)nwaves;\n  const uint32_t lt = 6u;\n")],
    # measurement: per-wave phase timestamps (s_memrealtime, 100 MHz) written
    # after the results: entry, descriptors in, tables in, first fold, ring
    # drained, exit (tools/direct_timeline.py reads them)
    "direct_ts": [
        ("crc32c_direct.hip", "  const uint32_t nwaves = gridDim.x * kDirectWaves;\n",
         "  const uint32_t nwaves = gridDim.x * kDirectWaves;\n"
         "  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();\n  uint64_t ts1 = 0, ts2 = 0, ts3 = 0, ts4 = 0, tsw = 0;\n"),
        ("crc32c_direct.hip", "    if (has_init) vinit = a.init[sbase + lane];\n  }\n",
         "    if (has_init) vinit = a.init[sbase + lane];\n  }\n"
         "  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n  ts1 = __builtin_amdgcn_s_memrealtime();\n"),
        ("crc32c_direct.hip", "    asm volatile(\"s_waitcnt lgkmcnt(0)\\n\\ts_barrier\" ::: \"memory\");\n",
         "    asm volatile(\"s_waitcnt lgkmcnt(0)\\n\\ts_barrier\" ::: \"memory\");\n"
         "    ts2 = __builtin_amdgcn_s_memrealtime();\n"),
        ("crc32c_direct.hip",
         "          if (tk[q].valid()) fold(tk[q], wb[q], eb[q]);\n",
         "          if (tsw == 0) tsw = __builtin_amdgcn_s_memrealtime();\n"
         "          if (tk[q].valid()) fold(tk[q], wb[q], eb[q]);\n"
         "          if (ts3 == 0) ts3 = __builtin_amdgcn_s_memrealtime();\n"),
        ("crc32c_direct.hip",
         "      for (int q = 0; q < 2; ++q) wait_task<0>(wb[q], eb[q]);\n    }\n",
         "      for (int q = 0; q < 2; ++q) wait_task<0>(wb[q], eb[q]);\n    }\n"
         "      ts4 = __builtin_amdgcn_s_memrealtime();\n"),
        ("crc32c_direct.hip", "    }\n  }\n\n}\n\nhipError_t launch_direct",
         "    }\n  }\n  if (a.out != nullptr && n >= 4096u && lane < 8u) {  // (not the self-test's 3-span calls: their out has no room)\n"
         "    const uint64_t ts5 = __builtin_amdgcn_s_memrealtime();\n"
         "    uint64_t v = lane == 0 ? ts0 : lane == 1 ? ts1 : lane == 2 ? ts2 : lane == 3 ? ts3 : lane == 4 ? ts4 :\n"
         "                 lane == 5 ? ts5 : lane == 6 ? (uint64_t)m : tsw;\n"
         "    reinterpret_cast<uint64_t*>(a.out + ((n + 3u) & ~3u))[8u * wave + lane] = v;\n  }\n}\n\nhipError_t launch_direct"),
    ] + MEASURE_ONLY,
    # the one-launch kernel before round 4's ring change: two slots of three
    # streams (the round-3 source, from git history)
    "ring6": [("crc32c_direct.hip", "@git", "bab2234:prismdb_amd/csrc/crc32c_direct.hip")],
    # round 4's first ring: one task sequence only, whatever the batch size
    "ring4": [("crc32c_direct.hip", "@git", "83d3f73:prismdb_amd/csrc/crc32c_direct.hip")],
    # two slots of two streams (positions mod 2): a fold waits for two tasks
    # and runs two LDS chains (a measurement copy kept in round 4's tree)
    "ring22": [("crc32c_direct.hip", "@git", "2cab585:tools/patches/crc32c_direct_ring22.hip")],
    # the ring before two single-task slots: four slots, and two task
    # sequences in pairs for short runs
    "slots4": [("crc32c_direct.hip", "@git", "8295f55:prismdb_amd/csrc/crc32c_direct.hip")],
    # the one-launch kernel at 16 waves per CU (1024-thread groups; needs
    # <= 128 VGPRs): fewer tasks per wave, so a wave's chain of folds ends sooner
    "w16": [("crc32c_device.h", "constexpr int kDirectThreads = 768;", "constexpr int kDirectThreads = 1024;")],
    # measurement-only (trailers not written): the one-launch kernel sealing
    # without its ring spans' trailer stores -- what they cost
    "noseal": [("crc32c_direct.hip",
                "        store_le32(reinterpret_cast<const uint8_t*>(hdr ? p - kLogCrcBack : body + gz + ((gf >> 12) & 3u)), res);\n",
                "        (void)p;\n        (void)body;\n")] + MEASURE_ONLY,
    # measurement-only (32 bytes around each trailer overwritten): the ring
    # spans' trailers stored as whole aligned 32-B sectors (two 16-B stores)
    # instead of one 4-B store -- whether partial-sector writes are the cost
    "sector32": [("crc32c_direct.hip",
                  "        store_le32(reinterpret_cast<const uint8_t*>(hdr ? p - kLogCrcBack : body + gz + ((gf >> 12) & 3u)), res);\n",
                  "        {\n"
                  "          const uint64_t ta = (hdr ? p - kLogCrcBack : body + gz + ((gf >> 12) & 3u)) & ~31ull;\n"
                  "          const u32x4 vv = {res, res, res, res};\n"
                  "          asm volatile(\"global_store_dwordx4 %0, %1, off\\n\\tglobal_store_dwordx4 %0, %1, off offset:16\"\n"
                  "                       : : \"v\"(ta), \"v\"(vv) : \"memory\");\n"
                  "        }\n")] + MEASURE_ONLY,
    # measurement-only, as sector32 but the whole aligned 64-B / 128-B line
    # around each trailer: does a full-line write spare the memory side a
    # fill of the line it merges a partial write into?
    "line64": [("crc32c_direct.hip",
                "        store_le32(reinterpret_cast<const uint8_t*>(hdr ? p - kLogCrcBack : body + gz + ((gf >> 12) & 3u)), res);\n",
                "        {\n"
                "          const uint64_t ta = (hdr ? p - kLogCrcBack : body + gz + ((gf >> 12) & 3u)) & ~63ull;\n"
                "          const u32x4 vv = {res, res, res, res};\n"
                "          asm volatile(\"global_store_dwordx4 %0, %1, off\\n\\tglobal_store_dwordx4 %0, %1, off offset:16\\n\\t\"\n"
                "                       \"global_store_dwordx4 %0, %1, off offset:32\\n\\tglobal_store_dwordx4 %0, %1, off offset:48\"\n"
                "                       : : \"v\"(ta), \"v\"(vv) : \"memory\");\n"
                "        }\n")] + MEASURE_ONLY,
    "line128": [("crc32c_direct.hip",
                 "        store_le32(reinterpret_cast<const uint8_t*>(hdr ? p - kLogCrcBack : body + gz + ((gf >> 12) & 3u)), res);\n",
                 "        {\n"
                 "          const uint64_t ta = (hdr ? p - kLogCrcBack : body + gz + ((gf >> 12) & 3u)) & ~127ull;\n"
                 "          const u32x4 vv = {res, res, res, res};\n"
                 "          asm volatile(\"global_store_dwordx4 %0, %1, off\\n\\tglobal_store_dwordx4 %0, %1, off offset:16\\n\\t\"\n"
                 "                       \"global_store_dwordx4 %0, %1, off offset:32\\n\\tglobal_store_dwordx4 %0, %1, off offset:48\\n\\t\"\n"
                 "                       \"global_store_dwordx4 %0, %1, off offset:64\\n\\tglobal_store_dwordx4 %0, %1, off offset:80\\n\\t\"\n"
                 "                       \"global_store_dwordx4 %0, %1, off offset:96\\n\\tglobal_store_dwordx4 %0, %1, off offset:112\"\n"
                 "                       : : \"v\"(ta), \"v\"(vv) : \"memory\");\n"
                 "        }\n")] + MEASURE_ONLY,
    # the lane kernel's 128-B line loads non-temporal (round 2 measured nt
    # halving the v2 kernel, whose tasks straddled lines; v3's are line-aligned)
    "lane_nt": [("crc32c_kernels.hip",
                 '    asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(w[J]) : "v"(addr), "n"(16 * J));\n',
                 '    asm volatile("global_load_dwordx4 %0, %1, off offset:%2 nt" : "=v"(w[J]) : "v"(addr), "n"(16 * J));\n')],
    # the trailer store before round 4's r04o (plain, no nt) -- against the product's nt
    "st_plain": [("crc32c_fold.h", '  asm volatile("global_store_dword %0, %1, off nt" : : "v"(p), "v"(v) : "memory");\n',
                  '  asm volatile("global_store_dword %0, %1, off" : : "v"(p), "v"(v) : "memory");\n')],
    # the lane kernel's log-header crc stores non-temporal too
    "lanest_nt": [("crc32c_kernels.hip",
                   '          asm volatile("global_store_dword %0, %1, off" : : "v"(ta), "v"(v) : "memory");\n',
                   '          asm volatile("global_store_dword %0, %1, off nt" : : "v"(ta), "v"(v) : "memory");\n')],
    # measurement-only bisection of the pair kernel against the fixed kernel
    # on the same blocks (valid for the sst3988 workload only: 3988-B spans at
    # stride 3992, init 0): records synthesized from the index, not read
    "pair_norec": [("crc32c_kernels.hip",
                    "    if (b < n) r = const_load(a.rec, b);\n    return r;\n  };\n"
                    "  auto make = [&](uint32_t b, const SpanRec& r, uint32_t first) -> PTask {\n",
                    "    if (b < n) {\n"
                    "      const uint64_t ad = reinterpret_cast<uint64_t>(a.base) + 3992ull * b;\n"
                    "      r.x = (uint32_t)ad;\n      r.y = ((uint32_t)(ad >> 32) & 0xffffu) | (27u << 16);\n"
                    "      r.z = 3988u;\n      r.w = 0xFFFFFFFFu;\n    }\n    return r;\n  };\n"
                    "  auto make = [&](uint32_t b, const SpanRec& r, uint32_t first) -> PTask {\n")] + MEASURE_ONLY,
    # ... and without the edge-byte load (no tail bytes, no verify there)
    "pair_noedge": [("crc32c_kernels.hip",
                     "    if (kVerify && lane >= 6u && lane < 10u) eoff = tl + (lane - 6u);\n    e = buf_ubyte(re, eoff);\n  };\n\n  uint32_t res = 0u, bad = 0u;\n",
                     "    if (kVerify && lane >= 6u && lane < 10u) eoff = tl + (lane - 6u);\n    (void)eoff;\n    e = 0u;\n  };\n\n  uint32_t res = 0u, bad = 0u;\n"),
                    ("crc32c_kernels.hip", "  constexpr int kYounger = 2 * (kRounds + 1);  // the other slot's two spans\n",
                     "  constexpr int kYounger = 2 * kRounds;  // the other slot's two spans\n")] + MEASURE_ONLY,
    # 16 waves per CU with the ticket path folding one chunk per step (its
    # two-chunk steps held 64 VGPRs): does the kernel then fit 128 VGPRs, and
    # do shorter runs per wave (~4 spans of a file instead of ~5.5) pay?
    "w16g1": [("crc32c_device.h", "constexpr int kDirectThreads = 768;", "constexpr int kDirectThreads = 1024;"),
              ("crc32c_direct.hip", "      constexpr int kG = 2;\n", "      constexpr int kG = 1;\n")],
    # WAL seal, measurement only (ignores neighbouring records' crc words in
    # the same sector): the lane kernel rewrites the whole aligned 32-B
    # sector holding a record's crc (loaded with the record's last task)
    # instead of one unaligned dword.  Does seal then reach verify?
    "walsec": [
        ("crc32c_kernels.hip",
         "__device__ __forceinline__ void wait_lane(u32x4 (&w)[8], uint32_t& hd, uint32_t& ed, uint32_t& sc, uint64_t& noff,\n"
         "                                          uint32_t& nlen, uint32_t& ninit) {\n"
         "  asm volatile(\"s_waitcnt vmcnt(8)\"\n"
         "               : \"+v\"(w[0]), \"+v\"(w[1]), \"+v\"(w[2]), \"+v\"(w[3]), \"+v\"(w[4]), \"+v\"(w[5]), \"+v\"(w[6]),\n"
         "                 \"+v\"(w[7]), \"+v\"(hd), \"+v\"(ed), \"+v\"(sc), \"+v\"(noff), \"+v\"(nlen), \"+v\"(ninit)\n",
         "__device__ __forceinline__ void wait_lane(u32x4 (&w)[8], uint32_t& hd, uint32_t& ed, uint32_t& sc, uint64_t& noff,\n"
         "                                          uint32_t& nlen, uint32_t& ninit, u32x4& sa, u32x4& sb) {\n"
         "  asm volatile(\"s_waitcnt vmcnt(8)\"\n"
         "               : \"+v\"(w[0]), \"+v\"(w[1]), \"+v\"(w[2]), \"+v\"(w[3]), \"+v\"(w[4]), \"+v\"(w[5]), \"+v\"(w[6]),\n"
         "                 \"+v\"(w[7]), \"+v\"(hd), \"+v\"(ed), \"+v\"(sc), \"+v\"(noff), \"+v\"(nlen), \"+v\"(ninit), \"+v\"(sa), \"+v\"(sb)\n"),
        ("crc32c_kernels.hip", "  uint64_t VP[2];\n  auto issue",
         "  uint64_t VP[2];\n  u32x4 SA[2] = {}, SB[2] = {};\n  auto issue"),
        ("crc32c_kernels.hip",
         "      if (kVerify) SC[sl] = asm_load_u32(owned && lastk ? (hdr ? vp - kLogCrcBack : vp + vlen) : zero);\n    }\n",
         "      if (kVerify) SC[sl] = asm_load_u32(owned && lastk ? (hdr ? vp - kLogCrcBack : vp + vlen) : zero);\n"
         "      if (!kVerify) {\n"
         "        const uint64_t sa = owned && lastk ? ((hdr ? vp - kLogCrcBack : vp + vlen) & ~31ull) : zero;\n"
         "        asm volatile(\"global_load_dwordx4 %0, %1, off\" : \"=v\"(SA[sl]) : \"v\"(sa));\n"
         "        asm volatile(\"global_load_dwordx4 %0, %1, off offset:16\" : \"=v\"(SB[sl]) : \"v\"(sa));\n"
         "      }\n    }\n"),
        ("crc32c_kernels.hip",
         "          asm volatile(\"global_store_dword %0, %1, off\" : : \"v\"(ta), \"v\"(v) : \"memory\");\n",
         "          const uint32_t b = (uint32_t)ta & 31u;\n"
         "          if (b > 28u) {\n"
         "            asm volatile(\"global_store_dword %0, %1, off\" : : \"v\"(ta), \"v\"(v) : \"memory\");\n"
         "          } else {\n"
         "            const uint32_t sh = 8u * (b & 3u), q = b >> 2;\n"
         "            const uint64_t v64 = (uint64_t)v << sh, m64 = 0xFFFFFFFFull << sh;\n"
         "            u32x4 s0 = SA[sl], s1 = SB[sl];\n"
         "            auto put = [&](uint32_t w, uint32_t d) -> uint32_t {\n"
         "              w = d == q ? (w & ~(uint32_t)m64) | (uint32_t)v64 : w;\n"
         "              return d == q + 1u ? (w & ~(uint32_t)(m64 >> 32)) | (uint32_t)(v64 >> 32) : w;\n"
         "            };\n"
         "            s0[0] = put(s0[0], 0); s0[1] = put(s0[1], 1); s0[2] = put(s0[2], 2); s0[3] = put(s0[3], 3);\n"
         "            s1[0] = put(s1[0], 4); s1[1] = put(s1[1], 5); s1[2] = put(s1[2], 6); s1[3] = put(s1[3], 7);\n"
         "            const uint64_t sa = ta & ~31ull;\n"
         "            asm volatile(\"global_store_dwordx4 %0, %1, off\" : : \"v\"(sa), \"v\"(s0) : \"memory\");\n"
         "            asm volatile(\"global_store_dwordx4 %0, %1, off offset:16\" : : \"v\"(sa), \"v\"(s1) : \"memory\");\n"
         "          }\n"),
        ("crc32c_kernels.hip", '"+v"(HD[0]), "+v"(ED[0]), "+v"(SC[0]) : : "memory");',
         '"+v"(HD[0]), "+v"(ED[0]), "+v"(SC[0]), "+v"(SA[0]), "+v"(SB[0]) : : "memory");'),
        ("crc32c_kernels.hip", "      wait_lane(W[sl], HD[sl], ED[sl], SC[sl], noff, nlen, ninit);\n",
         "      wait_lane(W[sl], HD[sl], ED[sl], SC[sl], noff, nlen, ninit, SA[sl], SB[sl]);\n"),
        ("crc32c_kernels.hip", '    asm volatile("" : "+v"(HD[sl]), "+v"(ED[sl]), "+v"(SC[sl]));\n',
         '    asm volatile("" : "+v"(HD[sl]), "+v"(ED[sl]), "+v"(SC[sl]), "+v"(SA[sl]), "+v"(SB[sl]));\n'),
    ],
    # measurement-only (trailers not written): the pair-run kernel sealing
    # without its once-per-run trailer stores -- what they cost on bulk SST seals
    "pair_noseal": [("crc32c_kernels.hip",
                     "        if (seal && ta != 0u) store_le32(reinterpret_cast<const uint8_t*>(ta), res);\n",
                     "        (void)ta;\n")] + MEASURE_ONLY,
    # the pair kernel's trailer stores plain (no nt) / write-through (sc0 sc1)
    "pair_st_plain": [("crc32c_kernels.hip",
                       "        if (seal && ta != 0u) store_le32(reinterpret_cast<const uint8_t*>(ta), res);\n",
                       "        if (seal && ta != 0u) asm volatile(\"global_store_dword %0, %1, off\" : : \"v\"(ta), \"v\"(res) : \"memory\");\n")],
    "pair_st_sc": [("crc32c_kernels.hip",
                    "        if (seal && ta != 0u) store_le32(reinterpret_cast<const uint8_t*>(ta), res);\n",
                    "        if (seal && ta != 0u) asm volatile(\"global_store_dword %0, %1, off sc0 sc1\" : : \"v\"(ta), \"v\"(res) : \"memory\");\n")],
    # the one-launch kernel's static runs weighted by the wave's place in its
    # group (waves 0-3 / 4-7 / 8-11)
    "w543": [("crc32c_direct.hip", "constexpr uint32_t kRunWeight[3] = {8u, 7u, 6u};",
              "constexpr uint32_t kRunWeight[3] = {5u, 4u, 3u};")],
    "w654": [("crc32c_direct.hip", "constexpr uint32_t kRunWeight[3] = {8u, 7u, 6u};",
              "constexpr uint32_t kRunWeight[3] = {6u, 5u, 4u};")],
    "w765": [("crc32c_direct.hip", "constexpr uint32_t kRunWeight[3] = {8u, 7u, 6u};",
              "constexpr uint32_t kRunWeight[3] = {7u, 6u, 5u};")],
    # the one-launch ring raising the priority of waves with more ring spans
    # left (s_setprio 0-3 by spans not yet started, after every issue)
    "prio": [("crc32c_direct.hip",
              "          tk[q] = static_task(jc, tk[q ^ 1]);\n          issue(tk[q], wb[q], eb[q]);\n",
              "          tk[q] = static_task(jc, tk[q ^ 1]);\n          issue(tk[q], wb[q], eb[q]);\n"
              "          {\n"
              "            const uint32_t rem = (uint32_t)__popcll(shortm & (jc >= 64u ? 0ull : ~0ull << jc));\n"
              "            if (rem >= 3u) __builtin_amdgcn_s_setprio(3);\n"
              "            else if (rem == 2u) __builtin_amdgcn_s_setprio(2);\n"
              "            else if (rem == 1u) __builtin_amdgcn_s_setprio(1);\n"
              "            else __builtin_amdgcn_s_setprio(0);\n"
              "          }\n")],
}

# the previous commit's kernels (a git worktree under build/:
# `git worktree add --detach build/wt_head HEAD`)
VARIANTS["prev"] = [("@src", os.path.join(ROOT, "build", "wt_head", "prismdb_amd", "csrc"), None)]
# other checkouts (git worktree add build/wt_<rev> <rev>): round 5's product,
# and round 6's planner lead-in change alone
VARIANTS["r05"] = [("@src", os.path.join(ROOT, "build", "wt_0f74c91", "prismdb_amd", "csrc"), None)]
VARIANTS["r06_parity"] = [("@src", os.path.join(ROOT, "build", "wt_72d150e", "prismdb_amd", "csrc"), None)]
# walsafe: walsec + the neighbour check (flag bit 26 of the lane's meta)
VARIANTS["walsafe"] = [
    (f, o, n.replace("const uint64_t sa = owned && lastk ?", "const uint64_t sa = owned && lastk && ((vmeta >> 26) & 1u) ?")
            .replace("          if (b > 28u) {\n", "          if (!((meta >> 26) & 1u)) {\n"))
    for f, o, n in VARIANTS["walsec"]] + [
    ("crc32c_kernels.hip",
     "      vmeta = n4 | (q0 << 16) | (h << 21) | (tb << 23) | ((owned ? 1u : 0u) << 25);\n",
     "      vmeta = n4 | (q0 << 16) | (h << 21) | (tb << 23) | ((owned ? 1u : 0u) << 25);\n"
     "      {\n"
     "        const int src = (int)(((lane + 63u) & 63u) << 2);\n"
     "        const uint32_t plo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)noff);\n"
     "        const uint32_t phi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(noff >> 32));\n"
     "        const uint32_t plen = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)nlen);\n"
     "        const uint64_t pvp = base + ((uint64_t)phi << 32 | plo);\n"
     "        const uint64_t ta = vp - kLogCrcBack, sa = ta & ~31ull;\n"
     "        const uint32_t b = (uint32_t)ta & 31u;\n"
     "        const bool sec = hdr && owned && b <= 28u && sa + 32u <= vp + vlen &&\n"
     "                         (b == 0u || (lane != 0u && pvp <= sa && pvp + plen >= ta));\n"
     "        vmeta |= (sec ? 1u : 0u) << 26;\n"
     "      }\n"),
]
# measurement: the pair-run kernel's per-wave entry and exit times
# (s_memrealtime, 100 MHz) written after the results (tools/wave_timeline.py)
VARIANTS["pair_ts"] = [
    ("crc32c_kernels.hip",
     "  __shared__ uint32_t lds[kLdsWords];\n  const uint32_t tid = threadIdx.x;\n  load_tables(lds, a.tabs, tid);\n"
     "  __syncthreads();\n  const uint32_t lane = tid & 63u;\n",
     "  __shared__ uint32_t lds[kLdsWords];\n  const uint32_t tid = threadIdx.x;\n"
     "  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();\n  load_tables(lds, a.tabs, tid);\n"
     "  __syncthreads();\n  const uint32_t lane = tid & 63u;\n"),
    ("crc32c_kernels.hip",
     "  // the abandoned slot's loads retire while their registers are live\n#pragma unroll\n"
     "  for (int sl = 0; sl < 2; ++sl) {\n    wait_task<0>(wb[sl][0], eb[sl][0]);\n"
     "    wait_task<0>(wb[sl][1], eb[sl][1]);\n  }\n}\n",
     "  // the abandoned slot's loads retire while their registers are live\n#pragma unroll\n"
     "  for (int sl = 0; sl < 2; ++sl) {\n    wait_task<0>(wb[sl][0], eb[sl][0]);\n"
     "    wait_task<0>(wb[sl][1], eb[sl][1]);\n  }\n"
     "  if (a.out != nullptr && n >= 4096u && lane < 2u) {  // (not the self-test's small calls)\n"
     "    const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();\n"
     "    reinterpret_cast<uint64_t*>(a.out + ((n + 3u) & ~3u))[2u * wave + lane] = lane == 0u ? ts0 : ts1;\n"
     "  }\n}\n"),
] + MEASURE_ONLY
# SIMD-slot priority rotation: a wave's user priority (s_setprio) is
# (its age rank on its SIMD + runs done) mod 4, so over four runs every wave
# spends a run at every priority (the youngest wave of each SIMD otherwise
# trails: profiles/r05/r05d_pair_wave_timeline.json)
SETPRIO = (
    "          if (rot == 0u) __builtin_amdgcn_s_setprio(0);\n"
    "          else if (rot == 1u) __builtin_amdgcn_s_setprio(1);\n"
    "          else if (rot == 2u) __builtin_amdgcn_s_setprio(2);\n"
    "          else __builtin_amdgcn_s_setprio(3);\n")
VARIANTS["fixed_rot"] = [
    ("crc32c_kernels.hip",
     "  uint64_t cur = wave * kRun;  // first span of the pair being folded\n  if (cur >= n) return;\n",
     "  uint64_t cur = wave * kRun;  // first span of the pair being folded\n  if (cur >= n) return;\n"
     "  uint32_t rot = rfl((tid >> 6) >> 2);\n  {\n" + SETPRIO + "  }\n"),
    ("crc32c_kernels.hip",
     "        if (nxt >= n || (nxt & (kRun - 1u)) == 0) flush();\n",
     "        if (nxt >= n || (nxt & (kRun - 1u)) == 0) {\n          flush();\n          rot = (rot + 1u) & 3u;\n"
     + SETPRIO + "        }\n"),
]
# measurement: the fixed kernel's per-wave entry and exit (tools/wave_timeline.py --work fixed)
VARIANTS["fixed_ts"] = [
    ("crc32c_kernels.hip",
     "  const uint64_t n = a.n;\n  __shared__ uint32_t lds[kLdsWords];\n  const uint32_t tid = threadIdx.x;\n",
     "  const uint64_t n = a.n;\n  __shared__ uint32_t lds[kLdsWords];\n  const uint32_t tid = threadIdx.x;\n"
     "  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();\n"),
    ("crc32c_kernels.hip",
     "    for (int j = 0; j < K; ++j) asm volatile(\"\" : \"+v\"(ring[d][j]));\n  }\n}\n",
     "    for (int j = 0; j < K; ++j) asm volatile(\"\" : \"+v\"(ring[d][j]));\n  }\n"
     "  if (a.out != nullptr && n >= 4096u && lane < 2u) {  // (not the self-test's small calls)\n"
     "    const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();\n"
     "    reinterpret_cast<uint64_t*>(a.out + ((n + 3u) & ~3ull))[2u * wave + lane] = lane == 0u ? ts0 : ts1;\n"
     "  }\n}\n"),
] + MEASURE_ONLY
# measurement: the span kernel's per-wave entry and exit (tools/wave_timeline.py --work mixed)
VARIANTS["span_ts"] = [
    ("crc32c_kernels.hip",
     "  if (blockIdx.x * 2u * kWavesPerGroup >= K) return;\n\n\n  __shared__ uint32_t lds[kLdsWords];\n",
     "  if (blockIdx.x * 2u * kWavesPerGroup >= K) return;\n"
     "  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();\n\n  __shared__ uint32_t lds[kLdsWords];\n"),
    ("crc32c_kernels.hip",
     "  // fixed kernel's drain).  Every slice was stored when its last record retired.\n#pragma unroll\n"
     "  for (int sl = 0; sl < 2; ++sl) {\n    wait_task<0>(wb[sl][0], eb[sl][0]);\n"
     "    wait_task<0>(wb[sl][1], eb[sl][1]);\n  }\n}\n",
     "  // fixed kernel's drain).  Every slice was stored when its last record retired.\n#pragma unroll\n"
     "  for (int sl = 0; sl < 2; ++sl) {\n    wait_task<0>(wb[sl][0], eb[sl][0]);\n"
     "    wait_task<0>(wb[sl][1], eb[sl][1]);\n  }\n"
     "  if (a.out != nullptr && a.role == kRoleSpans && a.n_dev == nullptr && n >= 4096u && lane < 2u) {\n"
     "    const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();\n"
     "    reinterpret_cast<uint64_t*>(a.out + ((n + 3u) & ~3u))[2u * wave + lane] = lane == 0u ? ts0 : ts1;\n"
     "  }\n}\n"),
] + MEASURE_ONLY
# the span kernel's task-balanced slices: 32 per stream instead of 16
VARIANTS["slices32"] = [("crc32c_device.h", "constexpr uint32_t kSlicesPerStream = 16;",
                         "constexpr uint32_t kSlicesPerStream = 32;")]
# the span kernel's dynamic tail: rounds of slices claimed on demand
VARIANTS["tail0"] = [("crc32c_kernels.hip", "constexpr uint32_t kTailRounds = 12;", "constexpr uint32_t kTailRounds = 0;"),
                     ("crc32c_kernels.hip", "constexpr uint32_t kPairTailRounds = 16;",
                      "constexpr uint32_t kPairTailRounds = 0;")]
VARIANTS["base_aa"] = []
# measurement-only (wrong results): what the lane kernel's fold costs on its
# clean lines -- words XORed instead of folded (no LDS lookups)
VARIANTS["lane_nofold"] = [("crc32c_kernels.hip", "      for (int i = 0; i < 32; ++i) y = step256(lds, tab, y, w[i >> 2][i & 3]);\n",
                            "      for (int i = 0; i < 32; ++i) y ^= w[i >> 2][i & 3];\n")] + MEASURE_ONLY
VARIANTS["fixed_ts_rot"] = VARIANTS["fixed_ts"] + VARIANTS["fixed_rot"]
# measurement-only (wrong results): the lane kernel's side loads with every
# lane reading the wave's zero region -- what the remaining ones cost
VARIANTS["lane_sidezero"] = [
    ("crc32c_kernels.hip", "      HD[sl] = asm_load_u32(owned && t.k == 0 && vq0 == 0u && vh != 0u ? vp & ~3ull : zero);\n",
     "      HD[sl] = asm_load_u32(zero);\n"),
    ("crc32c_kernels.hip",
     "      if (kVerify && hdr) SC[sl] = asm_load_u32(owned && t.k == 0 && 4u * vq0 < vh + kLogCrcBack ? vp - kLogCrcBack : zero);\n",
     "      if (kVerify && hdr) SC[sl] = asm_load_u32(zero);\n"),
    ("crc32c_kernels.hip",
     "      ED[sl] = asm_load_u32(owned && lastk && vtb != 0u && (vqe & 31u) == 0u ? vp + vlen - 4u : zero);\n",
     "      ED[sl] = asm_load_u32(zero);\n")] + MEASURE_ONLY
# ... or without them at all, with and without the fold of clean lines
VARIANTS["lane_noside"] = [
    ("crc32c_kernels.hip", "      HD[sl] = asm_load_u32(owned && t.k == 0 && vq0 == 0u && vh != 0u ? vp & ~3ull : zero);\n",
     "      HD[sl] = 0u;\n"),
    ("crc32c_kernels.hip",
     "      if (kVerify && hdr) SC[sl] = asm_load_u32(owned && t.k == 0 && 4u * vq0 < vh + kLogCrcBack ? vp - kLogCrcBack : zero);\n",
     "      SC[sl] = 0u;\n"),
    ("crc32c_kernels.hip",
     "      ED[sl] = asm_load_u32(owned && lastk && vtb != 0u && (vqe & 31u) == 0u ? vp + vlen - 4u : zero);\n",
     "      ED[sl] = 0u;\n")] + MEASURE_ONLY
VARIANTS["lane_bare"] = VARIANTS["lane_noside"] + VARIANTS["lane_nofold"][:1]
VARIANTS["lane_noout"] =[("crc32c_kernels.hip", "        if (a.out != nullptr) __builtin_nontemporal_store(v, a.out + rec);\n",
                           "")] + MEASURE_ONLY
# the lane kernel at 12 / 16 waves per CU
VARIANTS["lane_w12"] = [("crc32c_kernels.hip", "constexpr uint32_t kLaneThreads = 512;", "constexpr uint32_t kLaneThreads = 768;")]
VARIANTS["lane_w16"] = [("crc32c_kernels.hip", "constexpr uint32_t kLaneThreads = 512;", "constexpr uint32_t kLaneThreads = 1024;")]
# the lane kernel before the partial-line mask (round 5's committed kernels)
VARIANTS["lane_r05"] = [("crc32c_kernels.hip", "@git", "7af4fee:prismdb_amd/csrc/crc32c_kernels.hip")]
# the lane path before the long-span list moved to the side stream (710a890)
VARIANTS["lane_710a"] = [(f, "@git", "710a890:prismdb_amd/csrc/" + f)
                         for f in ("crc32c_kernels.hip", "crc32c_capi.hip", "crc32c_device.h")]
# the sealing lane kernel issuing its side loads only with a run's first /
# last task, as the verify kernel does
VARIANTS["lane_seal_cond"] = [("crc32c_kernels.hip", "    constexpr bool kSideAlways = !kVerify;\n",
                               "    constexpr bool kSideAlways = false;\n")]
# the lane kernel with one task in flight per wave (every wait drains: the
# next task's loads go out only after the fold) at 8 / 12 / 16 waves per CU:
# do more waves hide the fold better than the two-slot ring?
LANE_W1 = [("crc32c_kernels.hip", '  asm volatile("s_waitcnt vmcnt(8)"\n               : "+v"(w[0])',
            '  asm volatile("s_waitcnt vmcnt(0)"\n               : "+v"(w[0])')]
VARIANTS["lane_w8_1"] = LANE_W1
VARIANTS["lane_w12_1"] = LANE_W1 + VARIANTS["lane_w12"]
VARIANTS["lane_w16_1"] = LANE_W1 + VARIANTS["lane_w16"]
# the lane kernel before zero-region chunks (the committed HEAD's kernels)
VARIANTS["lane_head"] = [("crc32c_kernels.hip", "@git", "HEAD:prismdb_amd/csrc/crc32c_kernels.hip")]
# the trailer pass (planner-path sealing): measurement-only (neighbouring
# bytes rewritten unguarded: wrong for spans < 32 B apart) -- each trailer
# written as the whole aligned 32-B sector(s) around it, read first, instead
# of one 4-B partial write: do full-sector writes beat the partial ones?
TRAIL_STORE = "    store_le32(t, res[i]);\n  }\n}\n"
TRAIL_LOOP = ("  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += step) {\n"
              "    const uint64_t off = kDesc ? a.off[i] : i * a.stride;\n"
              "    const uint32_t len = kDesc ? a.len[i] : a.len_c;\n"
              "    const uint8_t* t = hdr ? a.base + off - kLogCrcBack : a.base + off + len;\n"
              "    store_le32(t, res[i]);\n  }\n}\n")
VARIANTS["trail_sector"] = [("crc32c_kernels.hip", TRAIL_STORE,
    "    {\n"
    "      const uint64_t ta = reinterpret_cast<uint64_t>(t), s0 = ta & ~31ull, s1 = (ta + 3u) & ~31ull;\n"
    "      const uint32_t v = res[i];\n"
    "      for (uint64_t sa = s0; sa <= s1; sa += 32u) {\n"
    "        uint32_t w[8];\n"
    "        for (int k = 0; k < 8; ++k) w[k] = reinterpret_cast<const uint32_t*>(sa)[k];\n"
    "        for (int k = 0; k < 8; ++k) {\n"
    "          const int64_t d = (int64_t)(sa + 4u * k) - (int64_t)ta;  // word k's offset from the trailer\n"
    "          uint64_t x = (uint64_t)w[k];\n"
    "          for (int b = 0; b < 4; ++b) {\n"
    "            const int64_t j = d + b;\n"
    "            if (j >= 0 && j < 4) x = (x & ~(0xFFull << (8 * b))) | ((uint64_t)((v >> (8 * j)) & 0xFFu) << (8 * b));\n"
    "          }\n"
    "          w[k] = (uint32_t)x;\n"
    "        }\n"
    "        typedef uint32_t v4t __attribute__((ext_vector_type(4)));\n"
    "        reinterpret_cast<v4t*>(sa)[0] = v4t{w[0], w[1], w[2], w[3]};\n"
    "        reinterpret_cast<v4t*>(sa)[1] = v4t{w[4], w[5], w[6], w[7]};\n"
    "      }\n"
    "    }\n  }\n}\n")] + MEASURE_ONLY
# the trailer pass in 128-thread blocks (twice the blocks)
VARIANTS["trail_b128"] = [("crc32c_kernels.hip",
    "  const uint64_t blocks = (a.n + 255u) / 256u;\n  const int grid = (int)(blocks < 16384u ? blocks : 16384u);\n"
    "  if (desc) crc32c_trailer_kernel<true><<<grid, 256, 0, s>>>(a, res);\n"
    "  else crc32c_trailer_kernel<false><<<grid, 256, 0, s>>>(a, res);\n",
    "  const uint64_t blocks = (a.n + 127u) / 128u;\n  const int grid = (int)(blocks < 32768u ? blocks : 32768u);\n"
    "  if (desc) crc32c_trailer_kernel<true><<<grid, 128, 0, s>>>(a, res);\n"
    "  else crc32c_trailer_kernel<false><<<grid, 128, 0, s>>>(a, res);\n")]
# batch_multi without its per-call timing events (t0 / t1 / t2 on the clique
# streams; prismdb_crc32c_multi_timing then reports nothing) -- what they cost
VARIANTS["multi_notime"] = [
    ("crc32c_multi.hip", "    if ((e = hipEventRecord(c->t0[p], c->streams[p])) != hipSuccess) return finish(HipFail(e, \"hipEventRecord\"));\n", ""),
    ("crc32c_multi.hip", "    if ((e = hipEventRecord(c->t1[p], c->streams[p])) != hipSuccess) return finish(HipFail(e, \"hipEventRecord\"));\n", ""),
    ("crc32c_multi.hip", "    if ((e = hipEventRecord(c->t2[p], c->streams[p])) != hipSuccess) return finish(HipFail(e, \"hipEventRecord\"));\n", ""),
    ("crc32c_multi.hip", "  c->timed = true;\n", "")]
# batch_multi with one device run straight on the caller's stream (no clique
# stream hand-offs) -- what the hand-offs cost
VARIANTS["multi_direct1"] = [
    ("crc32c_multi.hip", "  Clique* c = nullptr;\n  int rc = GetClique(ndev, devices, &c);\n",
     "  if (ndev == 1) {\n"
     "    if ((e = hipSetDevice(devices[0])) != hipSuccess) return HipFail(e, \"hipSetDevice\");\n"
     "    const int r1 = n[0] == 0 ? 0 : leveldb_crc32c_batch(dev_base[0], dev_off[0], dev_len[0], dev_init != nullptr ? dev_init[0] : nullptr,\n"
     "                                      n[0], out0, mismatch0, flags, streams != nullptr ? streams[0] : nullptr);\n"
     "    (void)hipSetDevice(cur);\n    return r1;\n  }\n"
     "  Clique* c = nullptr;\n  int rc = GetClique(ndev, devices, &c);\n")]
# measurement: the lane kernel's per-wave entry and exit (tools/wave_timeline.py --work wal)
VARIANTS["lane_ts"] = [
    ("crc32c_kernels.hip", "  const uint32_t first = wave * 64u;\n  if (first >= n) return;\n",
     "  const uint32_t first = wave * 64u;\n  if (first >= n) return;\n  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();\n"),
    ("crc32c_kernels.hip",
     "    asm volatile(\"\" : \"+v\"(HD[sl]), \"+v\"(ED[sl]), \"+v\"(SC[sl]));\n  }\n  asm volatile(\"\" : \"+v\"(noff), \"+v\"(nlen), \"+v\"(ninit));\n}\n",
     "    asm volatile(\"\" : \"+v\"(HD[sl]), \"+v\"(ED[sl]), \"+v\"(SC[sl]));\n  }\n  asm volatile(\"\" : \"+v\"(noff), \"+v\"(nlen), \"+v\"(ninit));\n"
     "  if (a.out != nullptr && n >= 4096u && lane < 2u) {  // (not the self-test's small calls)\n"
     "    const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();\n"
     "    reinterpret_cast<uint64_t*>(a.out + ((n + 3u) & ~3u))[2u * wave + lane] = lane == 0u ? ts0 : ts1;\n"
     "  }\n}\n"),
] + MEASURE_ONLY
# the lane kernel's claimed tail of runs: none / 4 / 12 rounds (product: 8)
for _r in (0, 4, 12):
    VARIANTS[f"lane_tail{_r}"] = [("crc32c_kernels.hip", "constexpr uint32_t kLaneTailRounds = 8;",
                                   f"constexpr uint32_t kLaneTailRounds = {_r};")]
# the lane kernel without its priority rotation (now that its tail is claimed)
VARIANTS["lane_noprio"] = [
    ("crc32c_kernels.hip", "  uint32_t prio = rfl(tid >> 6) >> 2;\n  if (prio == 0u) __builtin_amdgcn_s_setprio(0);\n  else __builtin_amdgcn_s_setprio(1);\n",
     "  uint32_t prio = 0u;\n"),
    ("crc32c_kernels.hip", "      prio ^= 1u;\n      if (prio == 0u) __builtin_amdgcn_s_setprio(0);\n      else __builtin_amdgcn_s_setprio(1);\n",
     "      (void)prio;\n")]
# combinations
VARIANTS["w111"] = [("crc32c_direct.hip", "constexpr uint32_t kRunWeight[3] = {8u, 7u, 6u};",
                     "constexpr uint32_t kRunWeight[3] = {1u, 1u, 1u};")]
VARIANTS["w765prio"] = VARIANTS["w765"] + VARIANTS["prio"]
VARIANTS["w654prio"] = VARIANTS["w654"] + VARIANTS["prio"]
VARIANTS["ts_w765"] = VARIANTS["direct_ts"] + VARIANTS["w765"]
VARIANTS["ts_w765prio"] = VARIANTS["direct_ts"] + VARIANTS["w765"] + VARIANTS["prio"]
# the one-launch kernel by a plain launch, its done event recorded after it
# (the product launches it with hipExtLaunchKernel and the event as its stop
# event): what the stop event does to a call's end (tools/percall_floor.py)
DIRECT_EXT = ("  if (verify)\n"
              "    hipExtLaunchKernelGGL(crc32c_direct_kernel<true>, dim3(grid), dim3(kDirectThreads), 0, s, nullptr, done, 0u, a, d);\n"
              "  else\n"
              "    hipExtLaunchKernelGGL(crc32c_direct_kernel<false>, dim3(grid), dim3(kDirectThreads), 0, s, nullptr, done, 0u, a, d);\n"
              "  return hipGetLastError();\n")
VARIANTS["direct_plain"] = [("crc32c_direct.hip", DIRECT_EXT,
                             "  if (verify)\n    crc32c_direct_kernel<true><<<grid, kDirectThreads, 0, s>>>(a, d);\n"
                             "  else\n    crc32c_direct_kernel<false><<<grid, kDirectThreads, 0, s>>>(a, d);\n"
                             "  hipError_t e = hipGetLastError();\n"
                             "  return e != hipSuccess ? e : hipEventRecord(done, s);\n")]
VARIANTS["direct_ts_plain"] = VARIANTS["direct_ts"] + VARIANTS["direct_plain"]
# the trailer pass's stores plain (write-back through L2) instead of
# non-temporal: 2.4 M scattered dword stores took the pass 117 us on a config-5
# call, the same stores from a bare kernel 38 us (tools/trailer_probe.py)
# (lane_pass -- log-record seals through the trailer pass, -4 %,
# profiles/r06/r06o -- needs the lane path's scatter before the pass, which
# the sealing tail no longer runs since the pass moved ahead of the join)
# the non-temporal trailer pass with four spans per thread, loads first
VARIANTS["trail_nt4"] = [("crc32c_kernels.hip", TRAIL_LOOP,
    "  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < a.n; i0 += step * 4u) {\n"
    "    const uint8_t* t[4];\n    uint32_t v[4];\n"
    "#pragma unroll\n    for (uint32_t k = 0; k < 4u; ++k) {\n"
    "      const uint64_t i = i0 + k * step;\n      t[k] = nullptr;\n      v[k] = 0u;\n"
    "      if (i < a.n) {\n"
    "        const uint64_t off = kDesc ? a.off[i] : i * a.stride;\n"
    "        const uint32_t len = kDesc ? a.len[i] : a.len_c;\n"
    "        t[k] = hdr ? a.base + off - kLogCrcBack : a.base + off + len;\n        v[k] = res[i];\n      }\n    }\n"
    "#pragma unroll\n    for (uint32_t k = 0; k < 4u; ++k)\n      if (t[k] != nullptr) store_le32(t[k], v[k]);\n  }\n}\n"),
    ("crc32c_kernels.hip", "  const uint64_t blocks = (a.n + 255u) / 256u;\n  const int grid = (int)(blocks < 16384u ? blocks : 16384u);\n  if (desc) return launch_k(crc32c_trailer_kernel",
     "  const uint64_t blocks = (a.n + 1023u) / 1024u;\n  const int grid = (int)(blocks < 16384u ? blocks : 16384u);\n  if (desc) return launch_k(crc32c_trailer_kernel")]
# the sealing lane kernel's header store held back to the next slot's wait
# and issued right after it, before that slot's fold: the store's write
# acknowledgement sits in the in-order vmcnt, and issued at the end of the
# fold it was waited for by the very next counted wait (profiles/r06/r06p_wal_pmc:
# TCP pending stalls 2x verify's); here the fold's work overlaps it
VARIANTS["lane_st_late"] = [
    ("crc32c_kernels.hip", "  u32x4 W[2][8];\n",
     "  u32x4 W[2][8];\n  uint64_t st_ta = 0;\n  uint32_t st_v = 0u, st_pend = 0u;  // a header store held back (seal)\n"),
    ("crc32c_kernels.hip",
     "          const uint64_t ta = hdr ? VP[sl] - kLogCrcBack : VP[sl] + len;\n"
     '          asm volatile("global_store_dword %0, %1, off" : : "v"(ta), "v"(v) : "memory");\n',
     "          st_ta = hdr ? VP[sl] - kLogCrcBack : VP[sl] + len;\n          st_v = v;\n          st_pend = 1u;\n"),
    ("crc32c_kernels.hip",
     "      wait_lane(W[sl], HD[sl], ED[sl], SC[sl], noff, nlen, ninit);\n",
     "      wait_lane(W[sl], HD[sl], ED[sl], SC[sl], noff, nlen, ninit);\n"
     "      if (!kVerify && st_pend != 0u) {\n"
     '        asm volatile("global_store_dword %0, %1, off" : : "v"(st_ta), "v"(st_v) : "memory");\n'
     "        st_pend = 0u;\n      }\n"),
    ("crc32c_kernels.hip",
     'drained:\n  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n',
     'drained:\n  if (!kVerify && st_pend != 0u) asm volatile("global_store_dword %0, %1, off" : : "v"(st_ta), "v"(st_v) : "memory");\n'
     '  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n'),
]
# the library's own events (per-call done events, side-stream fork / join)
# made with hipEventDisableSystemFence / hipEventReleaseToDevice: their
# records and stop events release at agent scope, not system scope (no L2
# write-back at the end of every call)
def _ev_flags(extra):
    return [("crc32c_capi.hip", f"hipEventCreateWithFlags(&{v}, hipEventDisableTiming);",
             f"hipEventCreateWithFlags(&{v}, hipEventDisableTiming | {extra});")
            for v in ("w.done[0]", "w.done[1]", "w->fork", "w->join")]


VARIANTS["ev_nofence"] = _ev_flags("hipEventDisableSystemFence")
VARIANTS["ev_device"] = _ev_flags("hipEventReleaseToDevice")
# the plan kernel with its descriptor loads hoisted: each thread loads U
# spans' (off, len, init) before building any record (the loads of one step
# in flight together instead of one span's at a time)
def _plan_hoist(U):
    src = open(os.path.join(ROOT, "prismdb_amd", "csrc", "crc32c_kernels.hip")).read()
    a = src.index("  uint32_t mine = 0;  // <= tile/256 spans")
    b = src.index("  atomicAdd(&sum, (unsigned long long)mine);")
    old = src[a:b]
    new = old.replace(
        "  for (uint64_t i0 = lo; i0 < hi; i0 += kPlanThreads) {\n    const uint64_t i = i0 + threadIdx.x;\n",
        f"  for (uint64_t i00 = lo; i00 < hi; i00 += {U}u * kPlanThreads) {{\n"
        f"  uint64_t doff[{U}];\n  uint32_t dlen[{U}], dinit[{U}];\n"
        f"#pragma unroll\n  for (uint32_t u = 0; u < {U}u; ++u) {{\n"
        "    const uint64_t i = i00 + u * kPlanThreads + threadIdx.x;\n    doff[u] = 0;\n    dlen[u] = 0;\n    dinit[u] = 0;\n"
        "    if (i < hi) {\n      const uint64_t q = a.idx != nullptr ? a.idx[i] : i;\n"
        "      doff[u] = kDesc ? a.off[q] : q * a.stride;\n      dlen[u] = kDesc ? a.len[q] : a.len_c;\n"
        "      dinit[u] = kDesc ? (a.init != nullptr ? a.init[q] : 0u) : a.init_c;\n    }\n  }\n"
        f"#pragma unroll\n  for (uint32_t u = 0; u < {U}u; ++u) {{\n"
        "    const uint64_t i0 = i00 + u * kPlanThreads;\n    const uint64_t i = i0 + threadIdx.x;\n")
    new = new.replace("    const uint64_t q = a.idx != nullptr ? a.idx[i] : i;  // the caller's span\n"
                      "    const uint64_t off = kDesc ? a.off[q] : q * a.stride;\n"
                      "    const uint32_t len = kDesc ? a.len[q] : a.len_c;\n"
                      "    const uint32_t init = kDesc ? (a.init != nullptr ? a.init[q] : 0u) : a.init_c;\n",
                      "    const uint64_t off = doff[u];\n    const uint32_t len = dlen[u];\n    const uint32_t init = dinit[u];\n")
    assert new.count("doff[u]") == 3 and new != old
    new = new.rstrip("\n") + "\n  }\n"
    return [("crc32c_kernels.hip", old, new)]


VARIANTS["plan_x2"] = _plan_hoist(2)
VARIANTS["plan_x4"] = _plan_hoist(4)
# the pair-run kernel's claimed tail: 8 / 24 / 32 rounds (product: 16)
for _r in (8, 24, 32):
    VARIANTS[f"ptail{_r}"] = [("crc32c_kernels.hip", "constexpr uint32_t kPairTailRounds = 16;",
                               f"constexpr uint32_t kPairTailRounds = {_r};")]
# the lane kernel's claimed tail on the eight claim lines (kClaimLines)
# instead of one counter (claims still read at once)
VARIANTS["lane8"] = [
    ("crc32c_capi.hip", "    a.claim = &ws.counters->lane_claim;  // (zeroed with the counters above)\n",
     "    a.claim = &ws.counters->lane_claim;  // (zeroed with the counters above)\n"
     "    a.claims = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws.counters) + 256);\n"),
    ("crc32c_kernels.hip",
     "      if (lane == 0u) got = __hip_atomic_fetch_add(a.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
     "      nx = Rs + rfl(got);\n",
     "      const uint32_t cset = (blockIdx.x >> 3) & (kClaimLines - 1u);\n"
     "      if (lane == 0u) got = __hip_atomic_fetch_add(a.claims + kClaimLineWords * cset, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
     "      nx = Rs + cset + kClaimLines * rfl(got);\n"),
]
# the span kernel's claimed tail on the eight claim lines (claims still read
# at once): counter (group / 8) % 8 deals the tail slices Kst + c + 8 j
VARIANTS["span8"] = [
    ("crc32c_kernels.hip",
     "        if (lane == 0u) got = __hip_atomic_fetch_add(a.claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
     "        k = Kst + rfl(got);\n",
     "        const uint32_t cset = (blockIdx.x >> 3) & (kClaimLines - 1u);\n"
     "        if (lane == 0u) got = __hip_atomic_fetch_add(a.claims + kClaimLineWords * cset, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
     "        k = Kst + cset + kClaimLines * rfl(got);\n"),
]
# the one-launch limit raised from 2^17 spans to 196 608 (64 spans per wave
# at 12 waves x 256 CUs): 8-11 SST files per call in one launch instead of
# two windows (tools/files_per_call.py)
VARIANTS["direct196k"] = [("crc32c_device.h", "constexpr uint64_t kDirectMaxSpans = 1ull << 17;",
                           "constexpr uint64_t kDirectMaxSpans = 196608ull;")]
# (trail_plain was adopted in 15de4d0 -- plain stores, four spans per thread,
# variants trail_x1 / trail_nt there -- and reverted: its dirty lines cost the
# next call more than the pass saved, profiles/r06/r06n_variants.json)


def do_build(names):
    from prismdb_amd.build import CSRC, build

    os.makedirs(VDIR, exist_ok=True)
    for f in os.listdir(VDIR):  # only this build's variants ship with the next GPU call
        if f.startswith("lib_") and f.endswith(".so"):
            os.remove(os.path.join(VDIR, f))

    for name in names:
        if name not in VARIANTS:
            continue
        vroot = os.path.join(ROOT, "build", "variants", name)  # sources and objects stay out of the GPU snapshot
        src = os.path.join(vroot, "pkg", "csrc")
        if os.path.isdir(src):
            shutil.rmtree(src)
        spec = VARIANTS[name]
        srcdir = CSRC
        if spec and spec[0][0] == "@src":  # ("@src", directory, None): another checkout's sources
            srcdir, spec = spec[0][1], spec[1:]
        shutil.copytree(srcdir, src)
        inc = os.path.join(vroot, "include")
        if not os.path.exists(inc):
            os.symlink(os.path.join(ROOT, "include"), inc)
        for fname, old, new in spec:
            path = os.path.join(src, fname)
            if old == "@git":  # (fname, "@git", "rev:path"): the whole file as it was at a commit
                with open(path, "wb") as f:
                    f.write(subprocess.check_output(["git", "-C", ROOT, "show", new]))
                continue
            with open(path) as f:
                text = f.read()
            if text.count(old) != 1:
                raise SystemExit(f"variant {name}: patch for {fname} matches {text.count(old)} times")
            with open(path, "w") as f:
                f.write(text.replace(old, new))
        print(build(src_dir=src, obj_dir=os.path.join(vroot, "obj"), lib_path=os.path.join(VDIR, f"lib_{name}.so")))


def do_run(args, names):
    import numpy as np
    import torch

    from prismdb_amd import crc32c  # product lib: data generator

    dev = torch.device("cuda", 0)
    nblk = (args.gib << 30) // 4096
    buf = torch.empty(nblk * 4096, dtype=torch.uint8, device=dev)
    crc32c.fill_synthetic(buf, 0x5EED0001)
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    libs = {}
    for name in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"lib_{name}.so"), mode=os.RTLD_LOCAL)
        f = lib.leveldb_crc32c_batch_fixed
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        g = lib.leveldb_crc32c_batch
        g.restype = ctypes.c_int
        g.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        libs[name] = (f, g)
    out = torch.empty(nblk, dtype=torch.int32, device=dev)
    mm = torch.empty(nblk, dtype=torch.uint8, device=dev)
    off4k = torch.arange(nblk, dtype=torch.int64, device=dev) * 4096
    len4k = torch.full((nblk,), 4096, dtype=torch.int32, device=dev)
    rng = np.random.default_rng(0x5EED0003)
    ml = rng.choice([1024, 4096, 16384, 65536], size=(args.gib << 30) // 21760 // 2).astype(np.int64)
    mo = np.concatenate([[0], np.cumsum(ml)[:-1]])
    moff, mlen = torch.from_numpy(mo).to(dev), torch.from_numpy(ml.astype(np.int32)).to(dev)
    # WAL records (~1 KB, log format) tiled over the buffer, verified with LOG_HEADER
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_configs import build_log
    from prismdb_amd import log

    fb = 4 << 20
    nf = (args.gib << 30) // fb // 4
    img = build_log(rng, fb)
    hoff, hlen = log.scan(img)
    buf[:nf * fb].view(nf, fb).copy_(torch.from_numpy(img).to(dev))
    woff = torch.from_numpy(((np.arange(nf, dtype=np.int64)[:, None] * fb + hoff.astype(np.int64)[None, :]) + 6)
                            .reshape(-1)).to(dev)
    wlen = torch.from_numpy(np.tile(hlen.astype(np.int32) + 1, nf)).to(dev)
    nw = woff.numel()
    crc32c.batch(buf, woff, wlen, mask=True, trailer=True, log_header=True)  # log::Writer's header crcs
    wout = torch.empty(nw, dtype=torch.int32, device=dev)
    wmm = torch.empty(nw, dtype=torch.uint8, device=dev)
    # SST data blocks through descriptors: 3988-B spans (contents + type) at stride 3992
    ns = (args.gib << 30) // 3992 - 1
    soff = torch.arange(ns, dtype=torch.int64, device=dev) * 3992
    slen = torch.full((ns,), 3988, dtype=torch.int32, device=dev)
    sout = torch.empty(ns, dtype=torch.int32, device=dev)
    # huge spans: 256 x (64 MiB - 5 B) at odd offsets, 2048 segments each (split path + combine)
    nh = min(256, (args.gib << 30) // (64 << 20) - 1)
    hoff_ = torch.arange(nh, dtype=torch.int64, device=dev) * (64 << 20) + 1
    hlen_ = torch.full((nh,), (64 << 20) - 5, dtype=torch.int32, device=dev)
    hout = torch.empty(max(nh, 1), dtype=torch.int32, device=dev)
    h1len = torch.full((1,), (1 << 30) - 3, dtype=torch.int32, device=dev)
    al = rng.integers(0, 70000, size=(args.gib << 30) // 35000 // 2).astype(np.int64)
    ao = np.sort(rng.integers(0, (args.gib << 30) // 2 - 70001, size=len(al))).astype(np.int64)
    aoff, alen = torch.from_numpy(ao).to(dev), torch.from_numpy(al.astype(np.int32)).to(dev)
    # one SST file's worth (16 811 data blocks + the 486 977-B index span), the
    # granularity a compaction verifies at: per-call latency, 50 calls per timing
    nfd = 16811
    foff = torch.from_numpy(np.concatenate([np.arange(nfd, dtype=np.int64) * 3992, [nfd * 3992]])).to(dev)
    flen = torch.from_numpy(np.concatenate([np.full(nfd, 3988, dtype=np.int32), [486977]]).astype(np.int32)).to(dev)
    fout = torch.empty(nfd + 1, dtype=torch.int32, device=dev)
    fmm = torch.empty(nfd + 1, dtype=torch.uint8, device=dev)
    # seven such files in one call (the most one launch takes: 117 684 spans)
    f7 = nfd * 3992 + 486977 + 4 + 3
    f7off = torch.from_numpy(np.concatenate([np.arange(7, dtype=np.int64)[:, None] * f7 + np.concatenate(
        [np.arange(nfd, dtype=np.int64) * 3992, [nfd * 3992]])[None, :]]).reshape(-1)).to(dev)
    f7len = flen.repeat(7)
    f2n, f3n = 2 * (nfd + 1), 3 * (nfd + 1)  # two and three files: either side of the two-sequence limit
    f7out = torch.empty(7 * (nfd + 1), dtype=torch.int32, device=dev)
    f7mm = torch.empty(7 * (nfd + 1), dtype=torch.uint8, device=dev)
    calls = {"sst_c5_seal": 6, "wal": 3, "wal_seal": 3, "file_fixed": 50, "file_desc": 50, "file_seal": 50, "file_verify": 50, "tiny_desc": 50,
             "files7_seal": 10, "files7_verify": 10, "files2_seal": 20, "files2_verify": 20,
             "files3_seal": 20, "files3_verify": 20}
    work = {
        "fixed4k": (lambda n: libs[n][0](buf.data_ptr(), 4096, 4096, nblk, 0, out.data_ptr(), None, 0, sp),
                    nblk * 4100),
        "desc4k": (lambda n: libs[n][1](buf.data_ptr(), off4k.data_ptr(), len4k.data_ptr(), None, nblk,
                                        out.data_ptr(), None, 0, sp), nblk * 4112),
        "verify4k": (lambda n: libs[n][0](buf.data_ptr(), 4096, 4092, nblk, 0, out.data_ptr(), mm.data_ptr(), 0,
                                          sp), nblk * 4105),
        "mixed": (lambda n: libs[n][1](buf.data_ptr(), moff.data_ptr(), mlen.data_ptr(), None, len(ml),
                                       out.data_ptr(), None, 0, sp), int(ml.sum()) + 16 * len(ml)),
        "wal": (lambda n: libs[n][1](buf.data_ptr(), woff.data_ptr(), wlen.data_ptr(), None, nw,
                                     wout.data_ptr(), wmm.data_ptr(), 0x4, sp),
                int(hlen.sum() + len(hlen)) * nf + nw * (4 + 1 + 12)),
        # log::Writer's header crcs, sealed in place (the same bytes: the buffer does not change)
        "wal_seal": (lambda n: libs[n][1](buf.data_ptr(), woff.data_ptr(), wlen.data_ptr(), None, nw,
                                          wout.data_ptr(), None, 0x7, sp),
                     int(hlen.sum() + len(hlen)) * nf + nw * (4 + 4 + 12)),
        "sst3988": (lambda n: libs[n][1](buf.data_ptr(), soff.data_ptr(), slen.data_ptr(), None, ns,
                                         sout.data_ptr(), None, 0, sp), ns * (3988 + 4 + 12)),
        # the same blocks through the fixed kernel (stride 3992, 3988 B; bytes
        # counted as for sst3988, so the rates compare as times)
        "sst3988_fixed": (lambda n: libs[n][0](buf.data_ptr(), 3992, 3988, ns, 0, sout.data_ptr(), None, 0, sp),
                          ns * (3988 + 4 + 12)),
        # the same spans sealed (MASK | WRITE_TRAILER): the planner path's trailer stores
        "sst3988_seal": (lambda n: libs[n][1](buf.data_ptr(), soff.data_ptr(), slen.data_ptr(), None, ns,
                                              sout.data_ptr(), None, 0x3, sp), ns * (3988 + 4 + 12)),
        # config 5's per-device batch size: 2.4 M SST spans sealed in one call (planner path, short runs)
        "sst_c5_seal": (lambda n: libs[n][1](buf.data_ptr(), soff.data_ptr(), slen.data_ptr(), None, 2404116,
                                             sout.data_ptr(), None, 0x3, sp), 2404116 * (3988 + 4 + 12)),
        "huge64m": (lambda n: libs[n][1](buf.data_ptr(), hoff_.data_ptr(), hlen_.data_ptr(), None, nh,
                                         hout.data_ptr(), None, 0, sp), nh * ((64 << 20) - 5 + 16)),
        "adversarial": (lambda n: libs[n][1](buf.data_ptr(), aoff.data_ptr(), alen.data_ptr(), None, len(al),
                                             out.data_ptr(), None, 0, sp), int(al.sum()) + 16 * len(al)),
        # the first 2^17 spans of the mixed and the random batch: one launch of the one-launch kernel
        "mixed17": (lambda n: libs[n][1](buf.data_ptr(), moff.data_ptr(), mlen.data_ptr(), None, 1 << 17,
                                         out.data_ptr(), None, 0, sp), int(ml[:1 << 17].sum()) + 16 * (1 << 17)),
        "adv17": (lambda n: libs[n][1](buf.data_ptr(), aoff.data_ptr(), alen.data_ptr(), None, 1 << 17,
                                       out.data_ptr(), None, 0, sp), int(al[:1 << 17].sum()) + 16 * (1 << 17)),
        "file_fixed": (lambda n: libs[n][0](buf.data_ptr(), 3992, 3988, nfd, 0, fout.data_ptr(), None, 0, sp),
                       nfd * (3988 + 4)),
        "file_desc": (lambda n: libs[n][1](buf.data_ptr(), foff.data_ptr(), flen.data_ptr(), None, nfd + 1,
                                           fout.data_ptr(), None, 0, sp), nfd * (3988 + 16) + 486977 + 16),
        "file_seal": (lambda n: libs[n][1](buf.data_ptr(), foff.data_ptr(), flen.data_ptr(), None, nfd + 1,
                                           fout.data_ptr(), None, 0x3, sp), nfd * (3988 + 16) + 486977 + 16),
        "file_verify": (lambda n: libs[n][1](buf.data_ptr(), foff.data_ptr(), flen.data_ptr(), None, nfd + 1,
                                             fout.data_ptr(), fmm.data_ptr(), 0, sp), nfd * (3988 + 17) + 486977 + 17),
        "files7_seal": (lambda n: libs[n][1](buf.data_ptr(), f7off.data_ptr(), f7len.data_ptr(), None, 7 * (nfd + 1),
                                             f7out.data_ptr(), None, 0x3, sp), 7 * (nfd * (3988 + 16) + 486977 + 16)),
        "files7_verify": (lambda n: libs[n][1](buf.data_ptr(), f7off.data_ptr(), f7len.data_ptr(), None, 7 * (nfd + 1),
                                               f7out.data_ptr(), f7mm.data_ptr(), 0, sp),
                          7 * (nfd * (3988 + 17) + 486977 + 17)),
        "files2_seal": (lambda n: libs[n][1](buf.data_ptr(), f7off.data_ptr(), f7len.data_ptr(), None, f2n,
                                             f7out.data_ptr(), None, 0x3, sp), 2 * (nfd * (3988 + 16) + 486977 + 16)),
        "files2_verify": (lambda n: libs[n][1](buf.data_ptr(), f7off.data_ptr(), f7len.data_ptr(), None, f2n,
                                               f7out.data_ptr(), f7mm.data_ptr(), 0, sp),
                          2 * (nfd * (3988 + 17) + 486977 + 17)),
        "files3_seal": (lambda n: libs[n][1](buf.data_ptr(), f7off.data_ptr(), f7len.data_ptr(), None, f3n,
                                             f7out.data_ptr(), None, 0x3, sp), 3 * (nfd * (3988 + 16) + 486977 + 16)),
        "files3_verify": (lambda n: libs[n][1](buf.data_ptr(), f7off.data_ptr(), f7len.data_ptr(), None, f3n,
                                               f7out.data_ptr(), f7mm.data_ptr(), 0, sp),
                          3 * (nfd * (3988 + 17) + 486977 + 17)),
        # one span of 1 GiB - 3 B at an odd offset: the one-launch path's few-huge-spans case
        "one_huge": (lambda n: libs[n][1](buf.data_ptr(), hoff_.data_ptr(), h1len.data_ptr(), None, 1,
                                          hout.data_ptr(), None, 0, sp), (1 << 30) - 3 + 16),
        # one 4 KiB span: the per-call floor of the one-launch path
        "tiny_desc": (lambda n: libs[n][1](buf.data_ptr(), off4k.data_ptr(), len4k.data_ptr(), None, 1,
                                           fout.data_ptr(), None, 0, sp), 4096 + 16),
    }

    def timed(fn, n, k=1):  # mean of k back-to-back calls
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            rc = fn(n)
            assert rc == 0, (n, rc)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3 / k

    if args.work:
        work = {w: v for w, v in work.items() if w in args.work}
    res = {w: {n: [] for n in names} for w in work}
    agree = {}
    outs_of = {"wal": wout, "wal_seal": wout, "sst3988": sout, "sst3988_seal": sout, "sst_c5_seal": sout, "sst3988_fixed": sout, "huge64m": hout, "one_huge": hout, "file_fixed": fout,
               "file_desc": fout, "file_seal": fout, "files7_seal": f7out, "files7_verify": f7out, "files2_seal": f7out,
               "files2_verify": f7out, "files3_seal": f7out, "files3_verify": f7out,
               "file_verify": fout, "tiny_desc": fout}
    for w, (fn, _) in work.items():
        ref = None
        for n in names:
            o = outs_of.get(w, out)
            o.fill_(0)
            timed(fn, n)
            got = o.clone()
            if ref is None:
                ref = got
            agree[f"{w}:{n}"] = bool(torch.equal(ref, got))
        if w == "wal":
            agree["wal:no_mismatch"] = int(wmm.sum()) == 0
    # The order alternates every rep: a variant run right after another on the
    # same workload was measured up to 2 % faster than the same library run
    # first (an A/A run of one library under two names,
    # profiles/r01_variants_aa_position_bias.json), e.g. descriptor arrays left
    # in the 256 MB Infinity Cache by the first run.
    for rep in range(args.reps):
        for w, (fn, _) in work.items():
            for n in (names if rep % 2 == 0 else names[::-1]):
                res[w][n].append(timed(fn, n, calls.get(w, 1)))
    print(json.dumps({"gib": args.gib, "reps": args.reps, "agree": agree,
                      "results": {w: {n: {"GB/s_median": round(work[w][1] / statistics.median(v) / 1e9, 1),
                                          "ms_median": round(statistics.median(v) * 1e3, 4)}
                                      for n, v in r.items()} for w, r in res.items()}}, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--gib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--work", nargs="*", help="workloads to time (default: all)")
    args = ap.parse_args()
    names = args.only or list(VARIANTS)
    if args.mode == "build":
        do_build(names)
    else:
        do_run(args, names)


if __name__ == "__main__":
    main()
