// EXPERIMENT (not on the library's hot path): persistent producer / consumer exact-histogram multiclass update, with
// its harness tools/kexp/persist_exp.hip.  Bit-identical to the two-pass route on every harness case (logits, NaN /
// inf / tied rows, ignore_index, probabilities, both mis-speculations, u16 wrap at N = 131072) but measured 2.2x
// SLOWER at 65536 x 1000 bf16 (profiles/persist_curve_experiment.json): the consumer's 127 KiB of class histograms
// leave the producer half a CU (8 waves), and a 32-row tile then takes ~15 us per CU (two-pass row pass: two
// 64-KiB blocks per CU, ~8 us per tile per CU).  Kept for the record and for future hardware with more LDS.
//
// Why: the two-pass route (curve_hist_kernels.h) writes the whole batch as class-major 16-bit codes to HBM and reads
// it back in a second launch: 131 MB logits + 131 MB codes written + 131 MB codes read per 65536 x 1000 bf16 update,
// plus a kernel boundary that writes the row pass's dirty L2 lines back.  Here ONE persistent launch (one
// 1024-thread workgroup per CU, all resident) does both roles and hands the codes over through the Infinity Cache
// in row chunks:
// One 512-thread workgroup per CU (2 waves per SIMD, 256 VGPRs: the tile in flight, the next tile's prefetch and the
// codes of both row pairs stay in registers; at 1024 threads the 128-VGPR cap spilled).
//   * producer role — per chunk, each workgroup turns one 32-row tile of logits into codes (the exact arithmetic
//     of row_tile: softmax with expf's instruction sequence, correctly rounded quotient, RNE to the input dtype,
//     arg-max + confusion matrix, rare NaN / inf rows listed) and writes them class-major with write-through (sc1)
//     vector stores, then bumps the chunk's ready counter (agent-scope atomic, after every wave's vmcnt(0) and a
//     workgroup barrier: the hand-off of MI355X_MICROARCH.md "Workgroup dispatch ... visibility", table row 1);
//   * consumer role — each workgroup owns k = ceil(C / G) <= 4 classes and keeps their negative-score histograms
//     in LDS for the whole batch (u16 pairs: 4 x 8132 words = 127 KiB); per chunk it polls the ready counter (one
//     lane, sc1 loads), then reads its classes' codes with sc1 loads (L1 bypassed) into LDS atomics.  It consumes
//     chunk s - 1 after producing chunk s, so the wait for the slowest producer overlaps the next tile's loads.
//     Positives (one per row) never enter the hand-off: the producer marks that element skipped and keeps the row's
//     positive code in a per-row u16 scratch, which the same workgroup adds to the int64 bins once the batch's
//     mode verdict is known — so a mis-speculated round leaves nothing global to undo.
//   * end — every workgroup reads the batch's real normalisation mode (written by producers before they signal);
//     if the speculated one was right it finishes the rare rows of its classes, adds its LDS counts to the int64
//     histogram (plain read-modify-write: exclusive owner) and widens the occupied code range.  If the speculation
//     was wrong, every workgroup sees it, and the SAME launch runs a second round with the real mode (codes only,
//     rare rows into list 1: the FIXUP semantics of the two-pass route) before flushing.
// u16 bins: a bin can only wrap after 65536 counts; chunks that could reach that use returning LDS atomics and a
// per-workgroup wrap table (+65536 per wrap, added at flush), so counts stay exact for any batch size.
// Waits are bounded (spin limit with s_sleep): a launch whose workgroups are not all resident cannot hang the GPU; it
// raises the timeout flag instead (read by the host at compute()).
#pragma once

#include "curve_hist_kernels.h"

namespace tmx {

#ifndef TMX_PERSIST_TILE_PROF
#define TMX_PERSIST_TILE_PROF 0  // harness-only: per-tile producer stamps instead of per-chunk phase stamps
#endif
constexpr int kPThreads = 512;  // producer workgroup
constexpr int kCThreads = 256;  // consumer workgroup: one wave per SIMD beside the producer's two
constexpr int kPWaves = kPThreads / kWave;  // 8: two row pairs of the 32-row tile per wave (pairs w and w + 8)
constexpr int kPHistWords = 8132;          // u16 pairs: codes 0 .. 16263 >= 16256 (bf16 1.0) and 15360 (fp16 1.0)
constexpr int kPMaxClasses = 4;            // classes per workgroup
constexpr int kPImageWords = 512 * kSlots; // one 512-class half of a 32-row tile (32 KiB)
constexpr int kPWrapSlots = 16;
constexpr int kPMaxChunks = 46;
// control words (int32) after the 8 words of mode_state: ready[2][kPMaxChunks] (round 1 / round 2), then
constexpr int kPCtrlTicket = 2 * kPMaxChunks;      // 2 G arrivals (producers and consumers)
constexpr int kPCtrlTimeout = kPCtrlTicket + 1;    // sticky error word (read as a deferred check at compute)
constexpr int kPCtrlProdDone = kPCtrlTicket + 2;   // producers done with round 0 (verdict barrier among producers)
constexpr int kPCtrlWords = kPCtrlTicket + 4;
// Two kernels share every CU: the consumer workgroup (4 class histograms) and the producer workgroup (one 512-class
// LDS image of a tile).  130,368 + 32,784 B <= 163,840 B with 512-B allocation granules (130,560 + 33,280).
constexpr size_t kPConsumerLds = (size_t)kPMaxClasses * kPHistWords * 4 + (size_t)kPWrapSlots * 8 + 128;
constexpr size_t kPProducerLds = (size_t)kPImageWords * 4 + 16;
constexpr size_t kPLdsBytes = kPConsumerLds;
constexpr long long kPSpinLimit = 1 << 22;  // ~4M polls with s_sleep(2): far beyond any healthy wait

// buffer resource over a byte range (< 2^31 B): raw loads / stores with an explicit cache policy
__device__ __forceinline__ __amdgpu_buffer_rsrc_t p_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
using p_v4u = __attribute__((ext_vector_type(4))) unsigned int;
#ifndef TMX_PERSIST_STORE_POLICY
#define TMX_PERSIST_STORE_POLICY 16  // harness A/B only: 0 = plain stores (NOT a valid hand-off across XCDs)
#endif
constexpr int kSc1 = 16;  // CPol SC1 (agent-coherent: write-through / L1 bypass)

// Workgroup barrier for LDS hand-offs only.  __syncthreads() on gfx950 also waits for every outstanding global load
// and store (vmcnt(0)) of the wave, which would drain the next tile's prefetch and the write-through stores at every
// LDS round; this waits for LDS operations only.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct PersistArgs {
  const void* preds;
  const int64_t* target;
  int64_t n, n_pad;
  int C, k, G, nchunks, tpw;  // classes per workgroup, grid, chunks, tiles per workgroup per chunk
  int* mode;                  // [2]: speculated (used) mode, verdict of this batch
  int* state;                 // [6]: rare-row counts [2], (unused) ticket, ...
  int* ctrl;                  // [kPCtrlWords]
  int64_t ignore_index;
  bool has_ignore;
  uint32_t* codes;            // class-major scratch [C][n_pad] u16 (the hand-off buffer)
  int64_t* hist;              // [C][2][kCodes]
  int64_t* confmat;           // [C][C] or null
  int* err;                   // or null
  int* slow_rows;             // [2][n]
  int* code_range;            // [C][2] or null
  uint16_t* pos_code;         // [n]: code of each row's target class (0x8000 = none)
  long long* prof;            // optional [G][4 * kPMaxChunks + 4] wall-clock stamps (harness profiling), else null
};

__device__ __forceinline__ int p_spin_until(int* ctr, int target, int* timeout_flag) {
  long long it = 0;
  int v;
  while ((v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < target) {
    if (++it > kPSpinLimit) {
      __hip_atomic_store(timeout_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return 1;
}

// Codes of one row pair (rows r0, r0 + 1 of this wave) for a fixed mode; the same arithmetic as row_tile.
// code[8 g + j] = class 512 g + 8 lane + j, row r0 in the low half, r0 + 1 in the high half.
// SOFTMAX and ROUND2 are wave-uniform RUNTIME flags (scalar branches), not template parameters: one copy of this
// body in the kernel (four inlined instances made a 280 KB code object).
// ``pos_t[h]`` = the target class of row r0 + h when the row is kept and its target is a class (its positive code is
// extracted from the LDS image in p_store_tile), else -1.
template <typename T, int NG>
__device__ __forceinline__ void p_pair_codes(const uint4 (&raw)[2][2], int64_t tv, int tlane, int64_t r0, const PersistArgs& a, int nvec,
                                             uint32_t (&code)[8 * NG], int (&pos_t)[2], bool& saw_bad, const bool SOFTMAX, const bool ROUND2) {
  const int lane = threadIdx.x & (kWave - 1);
  const bool lo_ok = lane < nvec, hi_ok = lane + kWave < nvec;
  const int64_t n = a.n;
  const int C = a.C;
  auto target_of = [&](int i) -> int64_t {
    const uint64_t u = static_cast<uint64_t>(tv);
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), i);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), i);
    return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  const int64_t ta = target_of(tlane), tb = target_of(tlane + 1);
  const bool va = r0 < n && !(a.has_ignore && ta == a.ignore_index);
  const bool vb = r0 + 1 < n && !(a.has_ignore && tb == a.ignore_index);
  RowStat<NG> ra, rb;
  row_stat<T, NG>(raw[0], lo_ok, hi_ok, ra);
  row_stat<T, NG>(raw[1], lo_ok, hi_ok, rb);
  bool fa = __builtin_isfinite(ra.mx), fb = __builtin_isfinite(rb.mx);
  int ama = 0, amb = 0;
  if (!ROUND2) {
    ama = row_argmax<NG>(ra);
    amb = row_argmax<NG>(rb);
  }
  float sa = 0.f, sb = 0.f, ia = 0.f, ib = 0.f;
  if (SOFTMAX) {
    float acc_a = 0.f, acc_b = 0.f;
#pragma unroll
    for (int j = 0; j < 8 * NG; ++j) {
      ra.v[j] = exp_nonpos(ra.v[j] - ra.mx);
      rb.v[j] = exp_nonpos(rb.v[j] - rb.mx);
      acc_a += ra.v[j];
      acc_b += rb.v[j];
    }
    sa = wave_sum_uniform(acc_a);
    sb = wave_sum_uniform(acc_b);
    ia = 1.f / sa;
    ib = 1.f / sb;
    fa = fa && sa == sa;
    fb = fb && sb == sb;
  } else {
    fa = fa && __builtin_isfinite(wave_sum_uniform(ra.sum));
    fb = fb && __builtin_isfinite(wave_sum_uniform(rb.sum));
  }
  const bool slow_a = va && !fa, slow_b = vb && !fb;
  if (!ROUND2 && !saw_bad) {
    saw_bad = slow_a || slow_b || (va && ra.mx > 1.f) || (vb && rb.mx > 1.f);
    if (!saw_bad && (va || vb)) saw_bad = wave_min_uniform(__builtin_fminf(va ? ra.mn : INFINITY, vb ? rb.mn : INFINITY)) < 0.f;
  }
  const bool ka = va && fa, kb = vb && fb;
  const uint32_t keep = (ka ? 0x0000FFFFu : 0u) | (kb ? 0xFFFF0000u : 0u);
  const uint32_t setm = ~keep & 0x80008000u;
#pragma unroll
  for (int j = 0; j < 8 * NG; ++j) {
    uint32_t packed;
    if (SOFTMAX) {
      packed = __builtin_amdgcn_perm(rne_word<T>(div_rn(rb.v[j], sb, ib)), rne_word<T>(div_rn(ra.v[j], sa, ia)), 0x07060302u);
    } else {
      const uint32_t ca = raw_code<T>(raw_bits<T>(raw[0][j >> 3], j & 7));
      const uint32_t cb = raw_code<T>(raw_bits<T>(raw[1][j >> 3], j & 7));
      packed = ca | (cb << 16);
    }
    code[j] = (packed & keep) | setm;
  }
  pos_t[0] = (ka && ta >= 0 && ta < C) ? static_cast<int>(ta) : -1;
  pos_t[1] = (kb && tb >= 0 && tb < C) ? static_cast<int>(tb) : -1;
  if (lane == 0) {
    const int64_t tt[2] = {ta, tb};
    const int am[2] = {ama, amb};
    const bool keepv[2] = {ka, kb}, slowv[2] = {slow_a, slow_b}, validv[2] = {va, vb};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t t = tt[i];
      if (!ROUND2) {
        if (a.confmat != nullptr && keepv[i] && t >= 0 && t < C && am[i] < C) atomic_add_i64(a.confmat + t * C + am[i], 1);
        if (a.err != nullptr && validv[i] && (t < 0 || t >= C)) atomicOr(a.err, 1);
      }
      if (slowv[i]) {
        const int list = ROUND2 ? 1 : 0;
        const int slot = atomicAdd(a.state + list, 1);
        __hip_atomic_store(a.slow_rows + list * n + slot, static_cast<int>(r0 + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// LDS transposition of one tile (all 16 waves hold one pair each) and write-through stores of its class segments.
// The positive element of each row leaves the hand-off here: lane 0 of each wave reads its rows' target-class words
// from the image, keeps the row's code in pos_code and sets the element's skip bit before the stores.
template <int NG>
__device__ __forceinline__ void p_store_tile(const uint32_t (&code)[2][8 * NG], const int (&pos_t)[2][2], uint32_t* __restrict__ s_img,
                                             const PersistArgs& a, __amdgpu_buffer_rsrc_t codes_rs, int64_t tile) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int p = wave + pp * kPWaves;  // pair slot
#pragma unroll
      for (int j = 0; j < 8; ++j) s_img[(8 * lane + j) * kSlots + (p ^ (lane & (kSlots - 1)))] = code[pp][8 * g + j];
    }
    lds_barrier();
    if (lane < 4) {  // lanes 0..3: (pair pp, row h) of this wave
      const int pp = lane >> 1, h = lane & 1;
      const int t = lane == 0 ? pos_t[0][0] : lane == 1 ? pos_t[0][1] : lane == 2 ? pos_t[1][0] : pos_t[1][1];  // no dynamic index
      const int64_t r = tile * kTileRows + 2 * (wave + pp * kPWaves) + h;
      if (t >= 0 && (t >> 9) == g) {
        const int cl = t & 511;
        const int idx = cl * kSlots + ((wave + pp * kPWaves) ^ ((cl >> 3) & (kSlots - 1)));
        const uint32_t wd = s_img[idx];
        a.pos_code[r] = static_cast<uint16_t>(h ? (wd >> 16) : (wd & 0xFFFFu));
        atomicOr(&s_img[idx], h ? 0x80000000u : 0x00008000u);  // both rows of a pair may share the word
      } else if (t < 0 && g == 0 && r < a.n) {
        a.pos_code[r] = 0x8000u;
      }
    }
    lds_barrier();
    constexpr int kQuads = kSlots / 4;
#pragma unroll
    for (int u = 0; u < 512 * kQuads / kPThreads; ++u) {
      const int idx = threadIdx.x + u * kPThreads;
      const int cl = idx / kQuads, q = idx % kQuads;
      const int c = 512 * g + cl;
      const int sw = (cl >> 3) & (kSlots - 1);
      const uint4 w = *reinterpret_cast<const uint4*>(&s_img[cl * kSlots + 4 * (q ^ (sw >> 2))]);
      const int x = sw & 3;
      const uint32_t e0 = x & 1 ? w.y : w.x, e1 = x & 1 ? w.x : w.y, e2 = x & 1 ? w.w : w.z, e3 = x & 1 ? w.z : w.w;
      const p_v4u o = x & 2 ? p_v4u{e2, e3, e0, e1} : p_v4u{e0, e1, e2, e3};
      if (c < a.C) {
        const uint32_t off = static_cast<uint32_t>((int64_t)c * a.n_pad * 2 + tile * (kTileRows * 2) + q * 16);
        __builtin_amdgcn_raw_buffer_store_b128(o, codes_rs, off, 0, TMX_PERSIST_STORE_POLICY);
      }
    }
    lds_barrier();
  }
}

// Loads of one tile: this wave's two row pairs (rows 2 p, 2 p + 1 of the tile, p = wave and wave + 8), and the
// targets of those four rows (lane i < 4 holds row i's).
template <typename T, int NG>
__device__ __forceinline__ void p_load_tile(const PersistArgs& a, int64_t tile, int nvec, uint4 (&raw)[2][2][2], int64_t& tv) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int lq = lane < nvec ? lane : nvec - 1, hq = lane + kWave < nvec ? lane + kWave : nvec - 1;
  const T* preds = static_cast<const T*>(a.preds);
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int64_t r0 = tile * kTileRows + 2 * (wave + pp * kPWaves);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint4* row = reinterpret_cast<const uint4*>(preds + min(r0 + h, a.n - 1) * a.C);
      raw[pp][h][0] = stream_load16(row + lq);
      if constexpr (NG == 2) raw[pp][h][1] = stream_load16(row + hq);
      else raw[pp][h][1] = raw[pp][h][0];
    }
  }
  tv = a.target[min(tile * kTileRows + 2 * (wave + ((lane & 3) >> 1) * kPWaves) + (lane & 1), a.n - 1)];
}

struct PConsumer {
  uint32_t* s_h;   // [kPMaxClasses][kPHistWords]
  uint32_t* s_wk;  // wrap table keys (class << 16 | bin), kPWrapSlots
  uint32_t* s_wc;  // wrap counts
  int* s_misc;     // [0] wrap slots used, [1] overflow-to-atomic flag
};

// Rare path (a 16-bit count wrapped): out of line, scalar arguments only, so it costs one call site per use instead
// of an unrolled 32-slot probe inlined at every LDS atomic.
__device__ __noinline__ void p_note_wrap(uint32_t* s_wk, uint32_t* s_wc, int* s_misc, int cls, int bin, int64_t* neg_hist_of_cls) {
  const uint32_t key = (static_cast<uint32_t>(cls) << 16) | static_cast<uint32_t>(bin);
#pragma unroll 1
  for (int i = 0; i < kPWrapSlots; ++i) {  // linear probe of a tiny table
    const uint32_t prev = atomicCAS(&s_wk[i], 0xFFFFFFFFu, key);
    if (prev == 0xFFFFFFFFu || prev == key) {
      atomicAdd(&s_wc[i], 1u);
      atomicMax(&s_misc[0], i + 1);
      return;
    }
  }
  atomic_add_i64(neg_hist_of_cls + bin, 65536);  // table full: straight to the bins; flush then adds atomically
  atomicOr(&s_misc[1], 1);
}

// Consume rows [rb, re) (multiple of 8) of this workgroup's classes from the hand-off buffer.
__device__ __forceinline__ void p_consume(const PersistArgs& a, const PConsumer& pc, __amdgpu_buffer_rsrc_t codes_rs, int c0, int kc,
                                          int64_t rb, int64_t re, const bool RTN) {
  const int64_t nv = (re - rb) / 8;  // uint4 per class
  const int64_t total = nv * kc;
  for (int64_t base = 0; base < total; base += 4 * kCThreads) {
    p_v4u w[4];
    int cls[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = base + threadIdx.x + u * kCThreads;
      cls[u] = -1;
      w[u] = p_v4u{0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};
      if (i < total) {
        cls[u] = static_cast<int>(i / nv);
        const int64_t v = i % nv;
        const uint32_t off = static_cast<uint32_t>((int64_t)(c0 + cls[u]) * a.n_pad * 2 + rb * 2 + v * 16);
        w[u] = __builtin_amdgcn_raw_buffer_load_b128(codes_rs, off, 0, kSc1);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (cls[u] < 0) continue;
      uint32_t* h = pc.s_h + cls[u] * kPHistWords;
      const uint32_t parts[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t x = (e & 1) ? (parts[e >> 1] >> 16) : (parts[e >> 1] & 0xFFFFu);
        if (x & 0x8000u) continue;  // skipped, or the row's positive (pos_code)
        const uint32_t code = x & 0x3FFFu;
        const uint32_t inc = (code & 1u) ? 0x10000u : 1u;
        if (RTN) {
          const uint32_t old = atomicAdd(&h[code >> 1], inc);
          const uint32_t half = (code & 1u) ? (old >> 16) : (old & 0xFFFFu);
          if (half == 0xFFFFu) {  // this add wrapped the 16-bit count: undo the carry into the neighbour, note +65536
            if (!(code & 1u)) atomicAdd(&h[code >> 1], 0xFFFF0000u);
            p_note_wrap(pc.s_wk, pc.s_wc, pc.s_misc, cls[u], static_cast<int>(code), a.hist + ((int64_t)(c0 + cls[u]) * 2) * kCodes);
          }
        } else {
          atomicAdd(&h[code >> 1], inc);
        }
      }
    }
  }
}

// Add the LDS counts of this workgroup's classes to the int64 histogram (exclusive owner) and widen the code range.
__device__ __forceinline__ void p_flush(const PersistArgs& a, const PConsumer& pc, int c0, int kc, int* lo_hi /* [kc][2] LDS */) {
  const bool atomic_mode = __hip_atomic_load(&pc.s_misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
  const int used = min(pc.s_misc[0], kPWrapSlots);
  constexpr int kB = 8;  // words per thread per batch: up to 16 independent int64 read-modify-writes in flight
  for (int cl = 0; cl < kc; ++cl) {
    uint32_t* h = pc.s_h + cl * kPHistWords;
    int64_t* neg = a.hist + ((int64_t)(c0 + cl) * 2) * kCodes;
    int lo = kCodes, hi = -1;
    for (int base = threadIdx.x; base < kPHistWords; base += kB * kCThreads) {
      int64_t cnt[2 * kB], old[2 * kB];
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        const int i = base + u * kCThreads;
        const uint32_t w = i < kPHistWords ? h[i] : 0u;
        cnt[2 * u] = static_cast<int64_t>(w & 0xFFFFu);
        cnt[2 * u + 1] = static_cast<int64_t>(w >> 16);
        for (int s = 0; s < used; ++s) {  // wrapped bins of this word (usually none)
          const uint32_t key = pc.s_wk[s];
          if ((key >> 16) == static_cast<uint32_t>(cl) && ((key & 0xFFFFu) >> 1) == static_cast<uint32_t>(i))
            cnt[2 * u + (key & 1u)] += 65536ll * pc.s_wc[s];
        }
      }
      if (!atomic_mode) {
#pragma unroll
        for (int q = 0; q < 2 * kB; ++q) old[q] = cnt[q] ? neg[2 * (base + (q >> 1) * kCThreads) + (q & 1)] : 0;
      }
#pragma unroll
      for (int q = 0; q < 2 * kB; ++q) {
        if (cnt[q] == 0) continue;
        const int bin = 2 * (base + (q >> 1) * kCThreads) + (q & 1);
        lo = min(lo, bin);
        hi = max(hi, bin);
        if (atomic_mode) atomic_add_i64(neg + bin, cnt[q]);
        else neg[bin] = old[q] + cnt[q];
      }
#pragma unroll
      for (int u = 0; u < kB; ++u)
        if (base + u * kCThreads < kPHistWords) h[base + u * kCThreads] = 0u;
    }
    lo = wave_min_i32(lo);
    hi = wave_max_i32(hi);
    if ((threadIdx.x & (kWave - 1)) == 0 && hi >= 0) {
      atomicMin(&lo_hi[2 * cl], lo);
      atomicMax(&lo_hi[2 * cl + 1], hi);
    }
  }
}

// Tile bookkeeping shared by both roles (tiles of chunk s: s * tpw * G + j * G + w, j < tpw).
struct PTiles {
  int64_t ntiles, chunk_tiles;
  int G, tpw, w;
  __device__ __forceinline__ int64_t tile(int s, int j) const {
    const int64_t t = (int64_t)s * chunk_tiles + (int64_t)j * G + w;
    return t < min<int64_t>((int64_t)(s + 1) * chunk_tiles, ntiles) ? t : ntiles;
  }
  __device__ __forceinline__ int in_chunk(int s) const {
    return static_cast<int>(min<int64_t>((int64_t)(s + 1) * chunk_tiles, ntiles) - (int64_t)s * chunk_tiles);
  }
};

// The last of the 2 G workgroups (producers and consumers) resets the hand-off counters, the rare-row counts and
// rolls the speculation; every workgroup read all of them before taking its ticket.
__device__ __forceinline__ void p_ticket(const PersistArgs& a, int verdict) {
  if (__hip_atomic_fetch_add(a.ctrl + kPCtrlTicket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 2 * a.G - 1) {
    for (int i = 0; i < 2 * kPMaxChunks; ++i) a.ctrl[i] = 0;
    a.ctrl[kPCtrlTicket] = 0;
    a.ctrl[kPCtrlProdDone] = 0;
    a.state[0] = a.state[1] = 0;
    a.mode[0] = verdict;
    a.mode[1] = 0;
  }
}

// Producer role: one 512-thread workgroup per CU turns its tiles of each chunk into class-major codes (write-through
// stores) and signals the chunk.  Round 1 (mis-speculated batches only) recomputes the codes with the real mode once
// every producer has finished round 0 (the verdict is then final).  Finally it adds its rows' positive codes.
template <typename T, int NG>
__global__ void __launch_bounds__(kPThreads, 2) mc_persist_producer(PersistArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t p_lds[];
  uint32_t* s_img = p_lds;
  int* s_p = reinterpret_cast<int*>(p_lds + kPImageWords);  // [0] saw a probability-mode witness, [1] verdict
  const int w = blockIdx.x;
  const int C = a.C;
  const int nvec = C / 8;
  const PTiles tl{a.n_pad / kTileRows, (int64_t)a.tpw * a.G, a.G, a.tpw, w};
  const __amdgpu_buffer_rsrc_t codes_rs = p_rsrc(a.codes, static_cast<uint32_t>((int64_t)C * a.n_pad * 2));
  int* timeout = a.ctrl + kPCtrlTimeout;
  if (threadIdx.x < 2) s_p[threadIdx.x] = 0;
  const int used_mode = a.mode[0];  // previous batch's verdict (kernel-boundary ordered)
  lds_barrier();
  int verdict = used_mode;
  for (int round = 0; round < 2; ++round) {
    if (round == 1 && verdict == used_mode) break;
    const int mode_now = round == 0 ? used_mode : verdict;
    int* ready = a.ctrl + round * kPMaxChunks;
    bool saw_bad = false;
    uint4 raw[2][2][2];
    int64_t tv = 0;
    if (tl.tile(0, 0) < tl.ntiles) p_load_tile<T, NG>(a, tl.tile(0, 0), nvec, raw, tv);
    for (int s = 0; s < a.nchunks; ++s) {
      long long* pf = (a.prof != nullptr && round == 0 && threadIdx.x == 0) ? a.prof + (int64_t)w * (4 * kPMaxChunks + 4) : nullptr;
      if (pf) pf[4 * s] = wall_clock64();
      int produced = 0;
      for (int j = 0; j < a.tpw; ++j) {
        const int64_t tile = tl.tile(s, j);
        if (tile >= tl.ntiles) break;
        uint32_t code[2][8 * NG];
        int pos_t[2][2];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int64_t r0 = tile * kTileRows + 2 * (threadIdx.x / kWave + pp * kPWaves);
          p_pair_codes<T, NG>(raw[pp], tv, 2 * pp, r0, a, nvec, code[pp], pos_t[pp], saw_bad, mode_now != 0, round != 0);
        }
        // prefetch this chunk's next tile now; the next chunk's first is loaded after the hand-off below (whose
        // vmcnt(0) would otherwise wait for it)
        if (j + 1 < a.tpw && tl.tile(s, j + 1) < tl.ntiles) p_load_tile<T, NG>(a, tl.tile(s, j + 1), nvec, raw, tv);
        p_store_tile<NG>(code, pos_t, s_img, a, codes_rs, tile);
        ++produced;
      }
      if (round == 0 && saw_bad) s_p[0] = 1;  // benign race: any witness
      // hand-off (MI355X_MICROARCH.md table row 1): every wave's sc1 stores and slow-row words complete, one
      // workgroup barrier, then one agent-scope add by one lane (the verdict word first when this chunk saw a witness)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0 && produced > 0) {
        if (round == 0 && s_p[0] && __hip_atomic_load(a.mode + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
          __hip_atomic_store(a.mode + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __hip_atomic_fetch_add(ready + s, produced, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (pf) pf[4 * s + 1] = wall_clock64();
      if (s + 1 < a.nchunks && tl.tile(s + 1, 0) < tl.ntiles) p_load_tile<T, NG>(a, tl.tile(s + 1, 0), nvec, raw, tv);
    }
    if (round == 0) {
      // the verdict is final once every producer finished round 0 (each wrote it before its last signal)
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(a.ctrl + kPCtrlProdDone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        p_spin_until(a.ctrl + kPCtrlProdDone, a.G, timeout);
        s_p[1] = __hip_atomic_load(a.mode + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      lds_barrier();
      verdict = s_p[1];
    }
  }
  // positives of this workgroup's rows, with the final codes (pos_code was written by this workgroup's own lanes)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int tiles_mine = a.nchunks * a.tpw;
  for (int base = 0; base < tiles_mine * kTileRows; base += kPThreads) {
    const int idx = base + threadIdx.x;
    if (idx >= tiles_mine * kTileRows) break;
    const int slot = idx / kTileRows;
    const int64_t tile = tl.tile(slot / a.tpw, slot % a.tpw);
    if (tile >= tl.ntiles) continue;
    const int64_t r = tile * kTileRows + idx % kTileRows;
    if (r >= a.n) continue;
    const uint32_t x = a.pos_code[r];
    if (x & 0x8000u) continue;
    const int64_t t = a.target[r];
    atomic_add_i64(a.hist + (t * 2 + 1) * kCodes + (x & 0x3FFFu), 1);
    if (a.code_range != nullptr) {
      atomicMin(a.code_range + 2 * t, static_cast<int>(x & 0x3FFFu));
      atomicMax(a.code_range + 2 * t + 1, static_cast<int>(x & 0x3FFFu));
    }
  }
  if (threadIdx.x == 0) p_ticket(a, verdict);
}

// Consumer role: one workgroup per CU owns k = ceil(C / G) <= 4 classes: LDS histograms of their negative codes for
// the whole batch, chunk by chunk as producers signal them; then the rare rows of its classes, its share of the
// rare rows' confusion-matrix entries, the flush into the int64 histogram and the occupied code range.
template <typename T>
__global__ void __launch_bounds__(kCThreads, 1) mc_persist_consumer(PersistArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t p_lds[];
  PConsumer pc;
  pc.s_h = p_lds;
  pc.s_wk = p_lds + kPMaxClasses * kPHistWords;
  pc.s_wc = pc.s_wk + kPWrapSlots;
  pc.s_misc = reinterpret_cast<int*>(pc.s_wc + kPWrapSlots);  // [0] wrap slots used, [1] atomic flush, [2] verdict
  int* s_range = pc.s_misc + 4;                                // [kPMaxClasses][2]
  const int w = blockIdx.x;
  const int C = a.C;
  const int c0 = min(w * a.k, C), kc = min(a.k, C - c0);
  const PTiles tl{a.n_pad / kTileRows, (int64_t)a.tpw * a.G, a.G, a.tpw, w};
  const __amdgpu_buffer_rsrc_t codes_rs = p_rsrc(a.codes, static_cast<uint32_t>((int64_t)C * a.n_pad * 2));
  int* timeout = a.ctrl + kPCtrlTimeout;
  auto clear = [&]() {
    uint4* s4 = reinterpret_cast<uint4*>(pc.s_h);
    for (int i = threadIdx.x; i < kPMaxClasses * kPHistWords / 4; i += kCThreads) s4[i] = make_uint4(0, 0, 0, 0);
    if (threadIdx.x < kPWrapSlots) { pc.s_wk[threadIdx.x] = 0xFFFFFFFFu; pc.s_wc[threadIdx.x] = 0u; }
    if (threadIdx.x < 2) pc.s_misc[threadIdx.x] = 0;
  };
  clear();
  if (threadIdx.x < 2 * kPMaxClasses) s_range[threadIdx.x] = (threadIdx.x & 1) ? -1 : kCodes;
  const int used_mode = a.mode[0];
  lds_barrier();
  int verdict = used_mode;
  for (int round = 0; round < 2; ++round) {
    if (round == 1) {
      if (verdict == used_mode) break;
      clear();  // mis-speculated: round 0 only touched LDS (positives wait in pos_code)
      lds_barrier();
    }
    int* ready = a.ctrl + round * kPMaxChunks;
    int64_t since_flush = 0;
    for (int s = 0; s < a.nchunks; ++s) {
      const int64_t rb = (int64_t)s * tl.chunk_tiles * kTileRows;
      const int64_t re = min<int64_t>((int64_t)(s + 1) * tl.chunk_tiles, tl.ntiles) * kTileRows;
      if (threadIdx.x == 0) p_spin_until(ready + s, tl.in_chunk(s), timeout);
      long long* pf = (a.prof != nullptr && round == 0 && threadIdx.x == 0) ? a.prof + (int64_t)w * (4 * kPMaxChunks + 4) : nullptr;
      if (pf) pf[4 * s + 2] = wall_clock64();
      lds_barrier();  // the poll's outcome; the payload loads are sc1 (table row 1: no acquire needed)
      if (kc > 0) p_consume(a, pc, codes_rs, c0, kc, rb, re, since_flush + (re - rb) > 65535);
      since_flush += re - rb;
      if (pf) pf[4 * s + 3] = wall_clock64();
    }
    if (round == 0) {
      if (threadIdx.x == 0) {
        pc.s_misc[2] = __hip_atomic_load(a.mode + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pc.s_misc[2] != used_mode && pc.s_misc[1]) __hip_atomic_store(timeout, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      lds_barrier();
      verdict = pc.s_misc[2];
    }
  }
  if (a.prof != nullptr && threadIdx.x == 0) a.prof[(int64_t)w * (4 * kPMaxChunks + 4) + 4 * kPMaxChunks] = wall_clock64();
  const bool fixed = verdict != used_mode;
  // rare rows (NaN / inf rows listed by producers) of this workgroup's classes: list 0 = speculated round, list 1 =
  // corrected round (fixed) — the class pass's rules (curve_hist_kernels.h class_hist_block)
  const int n0 = __hip_atomic_load(a.state + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int n1 = fixed ? __hip_atomic_load(a.state + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  const T* preds = static_cast<const T*>(a.preds);
  if (kc > 0 && n0 + n1 > 0) {
    for (int64_t i = threadIdx.x; i < (int64_t)(n0 + n1) * kc; i += kCThreads) {
      const int64_t li = i / kc;
      const int cl = static_cast<int>(i % kc);
      const int lst = li < n0 ? 0 : 1;
      if (lst == 0 && fixed) continue;
      const int r = __hip_atomic_load(a.slow_rows + lst * a.n + (lst == 0 ? li : li - n0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((lst == 1 ? verdict : used_mode) != 0) continue;  // softmax of a NaN / inf row: all NaN, every code skipped
      const int c = c0 + cl;
      const uint32_t code = raw_code<T>(bits16<T>(preds[(int64_t)r * C + c]));
      if (code & 0x8000u) continue;
      if (a.target[r] == c) {
        atomic_add_i64(a.hist + ((int64_t)c * 2 + 1) * kCodes + code, 1);
        atomicMin(&s_range[2 * cl], static_cast<int>(code));
        atomicMax(&s_range[2 * cl + 1], static_cast<int>(code));
      } else {
        const uint32_t old = atomicAdd(&pc.s_h[cl * kPHistWords + (code >> 1)], (code & 1u) ? 0x10000u : 1u);
        const uint32_t half = (code & 1u) ? (old >> 16) : (old & 0xFFFFu);
        if (half == 0xFFFFu) {
          if (!(code & 1u)) atomicAdd(&pc.s_h[cl * kPHistWords + (code >> 1)], 0xFFFF0000u);
          p_note_wrap(pc.s_wk, pc.s_wc, pc.s_misc, cl, static_cast<int>(code), a.hist + ((int64_t)c * 2) * kCodes);
        }
      }
    }
  }
  // confusion matrix of the listed rows of the speculated round (their arg-max: NaN first, else first maximum)
  if (a.confmat != nullptr && threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    for (int64_t i = w; i < n0; i += a.G) {
      const int64_t r = __hip_atomic_load(a.slow_rows + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t t = a.target[r];
      if (t < 0 || t >= C) continue;
      const T* row = preds + r * C;
      float best = -INFINITY;
      int bi = C, first_nan = C;
      for (int cc = lane; cc < C; cc += kWave) {
        const float v = to_f32<T>(row[cc]);
        if (v != v) first_nan = min(first_nan, cc);
        else if (bi == C || v > best) { best = v; bi = cc; }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) first_nan = min(first_nan, __shfl_xor(first_nan, off, kWave));
      wave_argmax(best, bi);
      const int am = first_nan < C ? first_nan : bi;
      if (lane == 0 && am < C) atomic_add_i64(a.confmat + t * C + am, 1);
    }
  }
  lds_barrier();
  if (kc > 0) {
    p_flush(a, pc, c0, kc, s_range);
    lds_barrier();
    if (a.code_range != nullptr && threadIdx.x < kc && s_range[2 * threadIdx.x + 1] >= 0) {
      atomicMin(a.code_range + 2 * (c0 + threadIdx.x), s_range[2 * threadIdx.x]);
      atomicMax(a.code_range + 2 * (c0 + threadIdx.x) + 1, s_range[2 * threadIdx.x + 1]);
    }
  }
  if (a.prof != nullptr && threadIdx.x == 0) a.prof[(int64_t)w * (4 * kPMaxChunks + 4) + 4 * kPMaxChunks + 1] = wall_clock64();
  if (threadIdx.x == 0) p_ticket(a, verdict);
}

// Host side: the launch geometry (grid = one workgroup per CU; None when the route does not apply).
struct PersistPlan {
  bool ok = false;
  int G = 0, k = 0, nchunks = 0, tpw = 0;
};

inline PersistPlan persist_plan(int64_t n, int C, int cus, int tpw_min = 1) {
  PersistPlan p;
  if (n <= 0 || C % 8 != 0 || C > 1024 || cus <= 0) return p;
  const int64_t n_pad = (n + kTileRows - 1) / kTileRows * kTileRows;
  if ((int64_t)C * n_pad * 2 >= (int64_t{1} << 31)) return p;  // 32-bit buffer offsets
  const int k = (C + cus - 1) / cus;
  if (k > kPMaxClasses) return p;
  const int64_t ntiles = n_pad / kTileRows;
  int64_t tpw = (ntiles + (int64_t)cus * kPMaxChunks - 1) / ((int64_t)cus * kPMaxChunks);
  if (tpw < tpw_min) tpw = tpw_min;
  const int64_t chunk_tiles = tpw * cus;
  p.G = cus;
  p.k = k;
  p.tpw = static_cast<int>(tpw);
  p.nchunks = static_cast<int>((ntiles + chunk_tiles - 1) / chunk_tiles);
  p.ok = p.nchunks <= kPMaxChunks;
  return p;
}

}  // namespace tmx
