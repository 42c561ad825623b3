// screen_x1.hip — single-term MFMA screen (fp16 host-rendered operands, bf16 device image) with lane-parallel batched threshold compaction.
//
// Same contract as screen_stream.hip (candidate ids per (query, slice), exact fp64 re-rank in
// refine.hip), different balance:
//
//  * ONE bf16 product per attribute (hi(q') * hi(x')), not the 3-term split: a third of the MFMA
//    work and half the fragment bytes.  The price is a wider error bound,
//        |a - a_exact| <= r1 * |q'| * max|x'| + r2 * max|x'|^2,
//    r1 ~ 2^-8 (bf16 rounding of both operands) — on the generate_input.py distribution that
//    lets ~2x k candidates through instead of ~k, which the exact re-rank absorbs easily.
//  * Candidate buffers hold 4-byte entries (top 16 bits of the fp32 4-row group max | 16-bit
//    slice-relative group index), so a wave's 64 columns x 64 entries fit in 17 KiB of LDS and
//    two waves share every SIMD (one wave's VALU epilogue overlaps the other's MFMAs).
//  * Threshold maintenance is batched and lane-parallel: when any lane's sub-buffer fills, the
//    whole wave compacts ALL 64 columns at once, lane j owning column j (per-lane radix select of
//    the k-th largest key over <= 64 register-resident entries).  The streaming kernel's
//    one-column-at-a-time ballot radix cost ~2.5k cycles per column; here a batch costs about as
//    much for all 64 columns, and every column's threshold rises at each batch.
//
// Element type: hl = 2 (prep.hip's device image) is bf16 hi/lo and runs v_mfma_f32_16x16x32_bf16;
// hl = 1 (host_prep.cpp's hi-only image and query fragments) is fp16 and runs
// v_mfma_f32_16x16x32_f16 at the same rate — 3 more significant bits per operand, a 4x tighter
// bound r1 (plus r3, the absolute error of fp16 subnormals), so fewer groups reach the re-rank.
//
// Layout (mfma_f32_16x16x32_bf16): lane (c = lane & 15, kg = lane >> 4) of column tile ct holds
// query column ct*16 + c and rows kg*4 .. kg*4+3 of the 16-point step.  The A operand (data
// fragments, hi half of prep.hip's hi/lo image) streams from L2 into a D-deep register ring; the
// C operand is the row's -|x'|^2/2, so acc = a directly.
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>

#include <cmath>

namespace {

// profiling: 1 no candidate path, 2 no epilogue (MFMA + loads only), 4 no norm loads (C = 0:
// wrong results, timing only), 8 event counters (g_x1_dbg), 32 / 64 fragment loads on every 2nd /
// 4th step only (the others reuse stale ring registers: wrong results, timing only — what a
// shared data ring would save on the texture path), 128 no hit after the first compaction (the
// threshold jumps to +inf: the step cost of a perfectly seeded threshold; profiles/r6c), 256
// per-lane exec-masked appends, 512 per-column-tile uniform append branches, 1024 the fill test
// at every taken step (the r9 form) instead of at the check points.  MODE 16
// is not an ablation: the
// COLLECT pass of the large-k pipeline (dmlp_screen_x1_collect)
int g_x1_mode = -1;  // -1: DMLP_X1_MODE (read once; default 0)
int x1_mode() {
  if (g_x1_mode < 0) {
    const char* e = getenv("DMLP_X1_MODE");
    g_x1_mode = e ? atoi(e) : 0;
  }
  return g_x1_mode;
}
__device__ unsigned long long g_x1_dbg[8];

// RING = 0: one wave per workgroup, each wave streams its slice's fragments from L2 into a
// register ring.  RING = R > 0: W = 8 waves per workgroup (one CU: 2 per SIMD), each with its own
// 64 query columns, share an R-tile LDS ring of the slice's fragments and C operands, filled by
// LDS-DMA (buffer_load ... lds): every tile crosses L2 -> CU once per workgroup instead of once
// per wave (the texture path ran ~90 % busy on per-wave loads: VERDICT r4, r5q/r7j profiles).
// The waves are not lock-stepped by barriers: each tile's 5 pieces (4 x 1 KiB of fragments + the
// 256-byte C operand) are issued by 5 of the 8 waves in rotation, a per-slot ready counter
// releases the tile and a per-slot done counter lets the slot be refilled, so one wave's
// compaction delays the others only once it falls RING - L tiles behind.
template <int KT, int SUB, int DEPTH, int CHECK, int CTV, int RING = 0>
struct X1Cfg {
  static constexpr int W = RING ? 8 : 1;        // waves per workgroup
  static constexpr int CT = CTV;                // MFMA column tiles per wave (4 or 8)
  static constexpr int NCOL = 16 * CT;          // queries per wave
  // column pitch in entries: 4 interleaved sub-buffers + 4 pad slots (which hold the 4
  // sub-buffer counts during a compaction); CP = 4 (mod 8) puts the 64 lanes of an append (16
  // columns x 4 sub-buffers, same fill) on 64 distinct banks
  static constexpr int CP = 4 * SUB + 4;
  // the fill check runs every CHECK steps, so a sub-buffer is compacted once it holds more than
  // SUB - CHECK entries (CHECK more appends always fit) and keeps at most SUB - CHECK of them
  static constexpr int CAPE = 4 * (SUB - CHECK);  // group entries a column may keep
  // group-id stride per (query, slice): the k class's (x1_sub: 16 or 32), any CHECK / ring SUB
  static constexpr int IDCAP = 4 * ((SUB <= 16 ? 16 : 32) - 1);
  static constexpr int SBUF = NCOL * CP * 4;
  // per wave without a ring: a 512-byte ring of two 4-step windows of the rows' -|x'|^2/2 (the
  // MFMA C operand), read with ds_read_b128 instead of a 16-byte-per-lane buffer load per step
  static constexpr int XRING = RING ? 0 : 512;
  static constexpr int TILEB = 4096 * KT;       // fragment bytes of a 64-point tile (hi only)
  static constexpr int RINGB = RING * (TILEB + 256);
  static constexpr int FLAGB = (2 * RING + 4) * 4;  // ready[R], done[R], fail
  static constexpr int LDS = W * SBUF + (RING ? RINGB + FLAGB : XRING);
  static constexpr int D = DEPTH;               // register-ring depth (steps in flight)
};

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// one 16x16x32 MFMA on 8 two-byte elements per lane: fp16 (F16) or bf16 bits
template <bool F16>
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// fp32 bits -> order-preserving u32 (only the top 16 bits are meaningful for a truncated key)
__device__ __forceinline__ unsigned ord32(unsigned b) {
  return b ^ ((unsigned)((int)b >> 31) | 0x80000000u);
}
__device__ __forceinline__ unsigned unord32(unsigned o) {
  return o ^ ((o >> 31) ? 0x80000000u : 0xffffffffu);
}

template <int KT, int SUB, int DEPTH, int CHECK, int CTV, int MODE, bool F16, int RING = 0>
__global__ __launch_bounds__(RING ? 512 : 64) __attribute__((amdgpu_waves_per_eu((CTV == 8 || SUB == 32 || KT >= 4) ? 1 : 2))) void k_screen_x1(
    const u32x4* __restrict__ xfrag, const f32x4* __restrict__ xinit4, int n_tiles, int n_points,
    const bf16x8* __restrict__ qhi, const float* __restrict__ qn, const int* __restrict__ qidx,
    const int* __restrict__ qk, int nq, const unsigned* __restrict__ xnmax_bits,
    const unsigned* __restrict__ bad, float r1, float r2, float r3, int S, int tiles_per_slice,
    int n_qblocks, int hl, int* __restrict__ cand_ids, int* __restrict__ cand_cnt,
    float* __restrict__ cand_h, const float* __restrict__ hseed, int ccap,
    const unsigned* __restrict__ rdy, int rdy_tiles, int rdy_n,
    const unsigned* __restrict__ xnm_sl, unsigned* __restrict__ estats, long long rdy_to,
    const unsigned* __restrict__ qrdy, int qrdy_q) {
  using C = X1Cfg<KT, SUB, DEPTH, CHECK, CTV, RING>;
  // COLLECT (large k, second pass): the threshold is fixed at the query's seed hseed[p] (a
  // lower bound on its k-th best score - 2 eps from the first pass); a full buffer is flushed to
  // the column's global list (up to ccap group entries per (query, slice)) instead of compacted
  constexpr bool COLLECT = (MODE & 16) != 0;
  static_assert(!(COLLECT && RING), "the COLLECT pass runs without the ring");
  constexpr int CT = C::CT;
  constexpr int D = C::D;
  constexpr int NH = C::NCOL / 64;  // columns per lane in the lane-owns-column phases
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wv = RING ? (int)(threadIdx.x >> 6) : 0;        // wave of the workgroup
  unsigned* const sbuf = (unsigned*)(smem + wv * C::SBUF);   // [col][CP] interleaved entries
  const unsigned sb0 = (unsigned)(wv * C::SBUF);             // its LDS byte offset

  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const int kg = lane >> 4;

  // ---- block -> (query block, slice); XCD-aware when S % 8 == 0 (slice s stays on one XCD's L2).
  // A ring workgroup's query block is W consecutive waves' columns.
  const int b = blockIdx.x;
  int qb, s;
  if ((S & 7) == 0) {
    const int xcd = b & 7, local = b >> 3, m = S >> 3;
    const int sl = local / n_qblocks;
    qb = local - sl * n_qblocks;
    s = xcd * m + sl;
  } else {
    s = b % S;
    qb = b / S;
  }
  const int t0 = s * tiles_per_slice;
  int t1 = t0 + tiles_per_slice;
  if (t1 > n_tiles) t1 = n_tiles;
  const int nt = t1 > t0 ? t1 - t0 : 0;
  const int nsteps = nt * 4;
  const int pbase = (qb * C::W + wv) * C::NCOL;

  if (*bad) {
    for (int col = lane; col < C::NCOL; col += 64)
      if (pbase + col < nq) cand_cnt[(int64_t)(pbase + col) * S + s] = -1;
    return;
  }
  // EARLY START (rdy != nullptr, S == 1): the data image is still crossing PCIe in rdy_n slices
  // of rdy_tiles tiles; rdy[i] turns nonzero once slice i (and its max norm xnm_sl[i]) landed.
  // The wave waits for a slice before its ring loads reach it, and a column's eps only covers
  // the slices scanned so far: it grows at each new slice (and its threshold drops by twice the
  // growth), so every compaction's bound holds for the entries it judges.  A wait that times
  // out (rdy_to ticks of the constant-rate wall clock, a few ms) marks the wave's queries
  // overflowed (the pipeline escalates them).  The ready word is written by a host-initiated copy:
  // it is polled with relaxed system-scope loads and followed by a system-scope acquire fence
  // before any image load.  Per wave: waits that had to spin, eps growths and timeouts go to
  // estats[0..2] at the end (the pipeline reports them).  With the LDS ring the wave that issues
  // a tile's pieces does the slice waits; every wave grows its eps as its scan reaches a slice.
  int have = 0;          // slices known landed (wave-uniform)
  bool rdy_fail = false;
  unsigned n_wait = 0, n_grow = 0, n_to = 0, n_qwait = 0;
  auto word_probe = [&](const unsigned* w) -> bool {
    unsigned* const f = const_cast<unsigned*>(w);
    return __builtin_amdgcn_readfirstlane(
               __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != 0u;
  };
  auto rdy_probe = [&](int i) -> bool { return word_probe(rdy + i); };
  auto wait_word = [&](const unsigned* w, unsigned& waits) -> bool {
    if (word_probe(w)) return true;
    ++waits;
    const long long t0 = wall_clock64();
    for (;;) {
      __builtin_amdgcn_s_sleep(2);
      if (word_probe(w)) return true;
      if (wall_clock64() - t0 > rdy_to) {
        ++n_to;
        return false;
      }
    }
  };
  auto wait_slice = [&](int i) -> bool { return wait_word(rdy + i, n_wait); };
  // m folded with the max norms of slices [lo, hi] (system-scope loads: ~1-2 us each, so the
  // words of slices already seen are not read again)
  auto fold_xnm = [&](float m, int lo, int hi) {
    for (int i = lo; i <= hi; ++i) {
      const unsigned* const f = xnm_sl + i;
      m = fmaxf(m, __uint_as_float(__hip_atomic_load(const_cast<unsigned*>(f), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM)));
    }
    return m;
  };
  // Once the last slice's word is set every slice has landed (the copies and their words run in
  // slice order on one stream): a wave that sees it takes the rest of the image at once instead
  // of probing slice by slice — each probe is a system-scope round trip on the wave's critical
  // path (the per-slice probes cost the screen ~0.075 ms: profiles/r7n_refine_ab.txt, r7s)
  auto widen = [&](int need) { return need < rdy_n - 1 && rdy_probe(rdy_n - 1) ? rdy_n - 1 : need; };

  // slice-local buffer resources: step j's fragments sit at j * KT * hl KiB (hi at +0, lo — when
  // the image carries it (hl = 2) — at +1 KiB per kt) and its -|x|^2/2 at j * 64 B, so the ring
  // loads need no address arithmetic beyond one scalar offset; prefetches past the slice read
  // zeros instead of faulting
  const int ks = hl * 1024;          // bytes between kt fragments of a step
  const int frags = 4 * KT * hl;     // 1 KiB fragments per 64-point tile
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(xfrag + (int64_t)t0 * (frags * 64)), (short)0, nt * frags * 64 * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(xinit4 + (int64_t)t0 * 16), (short)0, nt * 16 * 16, 0x00020000);

  // ---- the LDS ring (RING > 0): [R][TILEB] fragments | [R][256] C operands | ready[R] |
  // done[R] | fail | next.  ready[t % R] counts the published tiles of the slot (tile t is in
  // once it reaches t / R + 1); done[t % R] counts the waves that have read tile t out (slot t
  // may take tile t + R once it reaches 8 (t / R + 1)); next is the first tile nobody claimed.
  // A tile is claimed (compare-and-swap on next) by the first wave whose scan comes within L
  // tiles of it: that wave issues all its pieces (4 KT LDS-DMA fragments + the C operand) and
  // publishes it once its vmcnt drained — at its next tile, or before a compaction.  Every wait
  // is bounded (RTO); a timed-out wait sets fail and the workgroup's queries report overflow.
  constexpr int L = 3;
  constexpr int RS = RING > 0 ? RING : 1;  // (the per-wave variant never runs the ring code)
  constexpr long long RTO = 20000000;  // 200 ms of the 100 MHz wall clock: a bug, not a wait
  // The counters are plain LDS words with relaxed atomics: one wave's LDS operations execute in
  // issue order, so a counter read that returned before a wave's ring reads were issued orders
  // them (and a done increment issued after a wave's reads lands after them); a wavefront fence
  // keeps the compiler from moving the reads across.  An LDS-DMA piece is in LDS once the
  // issuing wave's vmcnt drained, before it publishes.
  constexpr unsigned ringA = (unsigned)(C::W * C::SBUF);
  constexpr unsigned ringN = ringA + (unsigned)(RING * C::TILEB);
  typedef __attribute__((address_space(3))) unsigned lds_u32;
  lds_u32* const rready = (lds_u32*)(size_t)(ringN + RING * 256);
  lds_u32* const rdone = rready + RING;
  lds_u32* const rfail = rdone + RING;
  lds_u32* const rnext = rfail + 1;
  typedef __attribute__((address_space(3))) void* lds_vp;
  auto lds_ld = [&](lds_u32* f) {
    return (unsigned)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
  };
  // spin until *f >= want (v: the value already read)
  auto lds_wait_v = [&](lds_u32* f, unsigned want, unsigned v) -> bool {
    if (v >= want) return true;
    const long long ts = wall_clock64();
    for (;;) {
      __builtin_amdgcn_s_sleep(1);
      if (lds_ld(f) >= want) return true;
      if (wall_clock64() - ts > RTO) {
        ++n_to;
        return false;
      }
    }
  };
  auto lds_wait = [&](lds_u32* f, unsigned want) { return lds_wait_v(f, want, lds_ld(f)); };
  auto ring_fail = [&]() {
    __hip_atomic_store(rfail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  int have_p = 0;  // slices this wave saw landed as a producer
  // claim tile t given nx, a read of next: true if this wave now owns its pieces
  auto claim_v = [&](int t, unsigned nx) -> bool {
    if (nx != (unsigned)t) return false;
    int got = 0;
    if (lane == 0) {
      unsigned e = (unsigned)t;
      got = __hip_atomic_compare_exchange_strong(rnext, &e, (unsigned)t + 1u, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return __builtin_amdgcn_readlane(got, 0) != 0;
  };
  auto claim = [&](int t) { return claim_v(t, lds_ld(rnext)); };
  // issue tile t's pieces into slot t % R (the claimer only)
  auto produce = [&](int t) {
    if (rdy && have_p < rdy_n) {
      const int si = min(t / rdy_tiles, rdy_n - 1);
      if (si >= have_p) {
        const int need = widen(si);
        bool ok = true;
        if (need == si)
          for (int i = have_p; i <= si && ok; ++i) ok &= wait_slice(i);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the host's DMA wrote them
        have_p = ok ? need + 1 : rdy_n;
        if (!ok) ring_fail();
      }
    }
    const int slot = t % RS;
    if (t >= RING && !lds_wait(rdone + slot, 8u * (unsigned)(t / RS))) ring_fail();
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            xr, (lds_vp)(smem + ringA + slot * C::TILEB + (p * KT + kt) * 1024), 16,
            lane * 16 + kt * ks, (t * 4 + p) * (KT * ks), 0, 0);
    if (lane < 16)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ir, (lds_vp)(smem + ringN + slot * 256), 16,
                                               lane * 16, t * 256, 0, 0);
  };
  auto publish = [&](int t) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's LDS-DMA pieces landed
    if (lane == 0)
      __hip_atomic_fetch_add(rready + t % RS, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto done_read = [&](int t) {  // this wave's reads of tile t are issued (LDS order retires them)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (lane == 0)
      __hip_atomic_fetch_add(rdone + t % RS, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  int pend = -1;  // the tile this wave issued and has not published yet

  float xnmax;
  if constexpr (RING > 0) {
    if (nsteps > 0) {
      if ((int)threadIdx.x < 2 * RING + 2) rready[threadIdx.x] = 0u;  // ready, done, fail, next
      __syncthreads();
      unsigned own = 0;
      for (int t = 0; t < L && t < nt; ++t)
        if (claim(t)) {
          produce(t);
          own |= 1u << t;
        }
      if (own) {
        __builtin_amdgcn_s_waitcnt(0x0F70);
        for (int t = 0; t < L && t < nt; ++t)
          if ((own >> t) & 1u) publish(t);
      }
    }
    // (a wave past the last query has no block to wait for)
    if (rdy && qrdy && pbase < nq) rdy_fail |= !wait_word(qrdy + pbase / qrdy_q, n_qwait);
    if (nsteps > 0 && !lds_wait(rready, 1u)) ring_fail();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (rdy) {  // slice 0 (at least) landed: a producer waited for it
      const int need = widen(0);
      xnmax = fold_xnm(0.0f, 0, need);
      have = need + 1;
    } else {
      xnmax = __uint_as_float(*xnmax_bits);
    }
  } else if (rdy) {
    // QUERY-BLOCK EARLY START (qrdy): the query operands cross PCIe in blocks of qrdy_q queries
    // (a multiple of the wave's columns), each with its own ready word: this wave waits only for
    // its own block before the prologue reads its queries' fragments and norms
    if (qrdy) rdy_fail |= !wait_word(qrdy + pbase / qrdy_q, n_qwait);
    // tiles 0..2: the prologue and step 0's loads
    const int need = widen(min(2 / rdy_tiles, rdy_n - 1));
    for (int i = 0; i <= need && !rdy_fail; ++i) rdy_fail |= !wait_slice(i);
    have = need + 1;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the host's DMA wrote them
    xnmax = fold_xnm(0.0f, 0, need);
  } else {
    xnmax = __uint_as_float(*xnmax_bits);
  }
  auto eps_of = [&](float qv, float xm) {
    return r1 * sqrtf(qv) * sqrtf(xm) + r2 * xm + r3 * (sqrtf(qv) + sqrtf(xm)) + r3 * 0x1p-15f;
  };

  bf16x8 bh[CT][KT];
  float h[CT];
  // per column tile: LDS byte address of this lane's next free slot (advances 16 B per append:
  // slots of one sub-buffer are 4 entries apart), and the address past which it must compact
  unsigned addr[CT], lim[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int p = pbase + ct * 16 + c;
    const bool valid = p < nq;
    const int q = valid ? qidx[p] : 0;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) bh[ct][kt] = qhi[(q * KT + kt) * 4 + kg];
    // COLLECT: a +inf seed marks a query whose first pass failed (it reports overflow; no real
    // seed is +inf).  (Not NaN: this file is built with -fno-honor-nans.)
    const float sd = COLLECT && valid ? hseed[p] : -FLT_MAX;
    const bool sbad = COLLECT && sd == INFINITY;
    h[ct] = valid && !sbad ? (COLLECT ? fmaxf(sd, -FLT_MAX) : -FLT_MAX) : INFINITY;
    addr[ct] = sb0 + (unsigned)(((ct * 16 + c) * C::CP + kg) * 4);
    lim[ct] = addr[ct] + (SUB - CHECK) * 16;
  }
  // per column in the lane-owns-column layout (lane j: column j + 64 hb): threshold, k, eps and
  // overflow flag, kept in registers; h[ct] above is the threshold in the MFMA layout (lane
  // c + 16 kg: column 16 ct + c), refreshed from oh by a lane shuffle
  float oh[NH], oe[NH];
  int okk[NH], ofl[NH];
#pragma unroll
  for (int hb = 0; hb < NH; ++hb) {
    const int p = pbase + lane + 64 * hb;
    const bool valid = p < nq;
    const int q = valid ? qidx[p] : 0;
    const float sd = COLLECT && valid ? hseed[p] : -FLT_MAX;
    const bool sbad = COLLECT && sd == INFINITY;
    oh[hb] = valid && !sbad ? (COLLECT ? fmaxf(sd, -FLT_MAX) : -FLT_MAX) : INFINITY;
    okk[hb] = valid ? qk[q] : 0;
    oe[hb] = valid ? eps_of(qn[q], xnmax) : 0.0f;
    ofl[hb] = sbad ? 1 : 0;
  }
  // h[ct] of the MFMA layout from the owners' oh
  auto pull_h = [&]() {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) h[ct] = __shfl(oh[ct >> 2], (ct & 3) * 16 + c);
  };

  // ---- batched compaction: lane j owns column j.  FINAL: write the column's candidate ids.
  // A column's entries are interleaved: slot s holds entry s >> 2 of sub-buffer s & 3, so the
  // lane reads its column as 16-byte vectors and re-deals the survivors by writing them back at
  // consecutive slots (slot s -> sub-buffer s & 3 again, i.e. round-robin).  The 4 sub-buffer
  // counts travel through the column's pad slots 4 SUB .. 4 SUB + 3.
  int nout[NH];  // COLLECT: group entries this lane's column has flushed so far
#pragma unroll
  for (int hb = 0; hb < NH; ++hb) nout[hb] = 0;
  auto compact = [&](const bool final_pass) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      sbuf[(ct * 16 + c) * C::CP + 4 * SUB + kg] =
          (addr[ct] - (lim[ct] - (SUB - CHECK) * 16)) >> 4;
    dmlp::wave_sync();
#pragma unroll 1
    for (int hb = 0; hb < NH; ++hb) {
    const int j = lane + 64 * hb;
    unsigned* const colbuf = sbuf + j * C::CP;
    const int4 n4 = *(const int4*)(colbuf + 4 * SUB);
    const int nm[4] = {n4.x, n4.y, n4.z, n4.w};
    if constexpr (COLLECT) {
      // flush: every buffered entry (appended at a group max >= the fixed seed) goes to the
      // column's global list as (ordered 16-bit key << 16 | slice-relative group index)
      const int pc = pbase + j;
      bool ov = ofl[hb] != 0;
      int no = nout[hb];
      int* const out = cand_ids + ((int64_t)pc * S + s) * ccap;
      if (pc < nq && !ov) {
#pragma unroll
        for (int v = 0; v < SUB; ++v) {
          const u32x4 raw = *(const u32x4*)(colbuf + 4 * v);
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            if (v < nm[m]) {
              if (no < ccap) out[no] = (int)((ord32(raw[m]) & 0xffff0000u) | (raw[m] & 0xffffu));
              ++no;
            }
          }
        }
        ov = no > ccap;
      }
      nout[hb] = no;
      if (!final_pass) {
        *(int4*)(colbuf + 4 * SUB) = int4{0, 0, 0, 0};
        if (ov) { oh[hb] = INFINITY; ofl[hb] = 1; }  // stop appending: the query overflowed
      } else if (pc < nq) {
        cand_cnt[(int64_t)pc * S + s] = ov ? -1 : no;
        cand_h[2 * ((int64_t)pc * S + s)] = oh[hb];
        cand_h[2 * ((int64_t)pc * S + s) + 1] = oe[hb];
      }
      continue;
    }
    const int kc = okk[hb];
    const float epc = oe[hb];
    const int flag = ofl[hb];
    float hc = oh[hb];
    // entries -> ordered keys in place (0 = empty slot)
    unsigned e[4 * SUB];
    // every buffered key is >= key(hc): appended at h = hc or kept at the last compaction
    unsigned mx = 0u;
    const unsigned mn = ord32(__float_as_uint(hc)) & 0xffff0000u;
#pragma unroll
    for (int v = 0; v < SUB; ++v) {
      const u32x4 raw = *(const u32x4*)(colbuf + 4 * v);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        // validity as arithmetic (all-ones iff v < count), not a predicate: 64 live lane masks
        // would spill SGPRs into the hot loop
        const unsigned vm = (unsigned)((v - nm[m]) >> 31);
        const unsigned o = ord32(raw[m]) & vm;
        e[4 * v + m] = o;
        mx = max(mx, o);
      }
    }
    const int ntot = nm[0] + nm[1] + nm[2] + nm[3];
    const bool sel = !flag && kc >= 1 && ntot >= kc;
    // k-th largest key, radix search below the common prefix of [min, max] on 15-bit keys
    // (key16 >> 1) packed two per register: one v_pk_sub_i16 / v_pk_lshrrev_b16 / v_pk_add_u16
    // triple counts two entries, with no VALU->SGPR->VALU carry chains.  Empty slots are 0 and
    // always count as "below".  2*T15 is then a (one-LSB) lower bound on the 16-bit k-th key.
    s16x2 pk[2 * SUB];
#pragma unroll
    for (int i = 0; i < 2 * SUB; ++i)
      pk[i] = __builtin_bit_cast(s16x2, (e[2 * i] >> 17) | ((e[2 * i + 1] >> 17) << 16));
    const unsigned dif = (mx ^ mn) >> 17;
    const int top = (sel && dif) ? 31 - __clz((int)dif) : -1;
    unsigned T = mx >> 17;
    if (top >= 0) T &= ~((2u << top) - 1u);
    int topw = top;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int t = __shfl_xor(topw, o);
      topw = t > topw ? t : topw;
    }
    for (int bit = topw; bit >= 0; --bit) {
      const short cand = (short)(T | (1u << bit));
      const s16x2 cc = {cand, cand};
      u16x2 lt = {0, 0};
#pragma unroll
      for (int i = 0; i < 2 * SUB; ++i) lt += __builtin_bit_cast(u16x2, pk[i] - cc) >> (unsigned short)15;
      const int ge = 4 * SUB - (int)lt.x - (int)lt.y;
      if (ge >= kc) T |= 1u << bit;
    }
    T <<= 1;  // back to the 16-bit key space (floor)
    if (sel) {
      // decode(T << 16) <= the k-th largest group max: a lower bound on the k-th best score
      const float ak = __uint_as_float(unord32(T << 16));
      hc = fmaxf(hc, ak - 2.0f * epc);
    }
    // keep every entry whose truncated key can be >= hc (floor(key) >= floor(key(hc))); hc >=
    // -FLT_MAX, so kh > 0 and empty slots (0) never pass; an overflowed column keeps nothing
    const unsigned kh = flag ? 0xffffffffu : ord32(__float_as_uint(hc)) & 0xffff0000u;
    if (MODE & 8) {
      if (lane == 0) atomicAdd(&g_x1_dbg[3], 1ull);
    }
    if (!final_pass) {
      int pos = 0;
#pragma unroll
      for (int i = 0; i < 4 * SUB; ++i) {
        const bool keep = e[i] >= kh;
        // every lane stores; a dropped entry lands in the next free slot (overwritten by the
        // next kept one, or past the new count: never read)
        colbuf[pos] = unord32(e[i]);
        pos += keep ? 1 : 0;
      }
      const bool ovf = flag || pos > C::CAPE;
      int4 nn;
      nn.x = ovf ? 0 : (pos + 3) >> 2;
      nn.y = ovf ? 0 : (pos + 2) >> 2;
      nn.z = ovf ? 0 : (pos + 1) >> 2;
      nn.w = ovf ? 0 : pos >> 2;
      *(int4*)(colbuf + 4 * SUB) = nn;
      oh[hb] = ovf ? INFINITY : hc;
      ofl[hb] = ovf ? 1 : 0;
    } else {
      // kept entries out as (ordered 16-bit key << 16 | slice-relative group index): the refine
      // takes the k-th largest key over ALL slices of the query (a global threshold, as tight as
      // one slice), then keeps the members whose recomputed single-term score reaches it
      const int p = pbase + j;
      if (p < nq) {
        int* const out = cand_ids + ((int64_t)p * S + s) * C::IDCAP;
        int kept = 0;
#pragma unroll
        for (int i = 0; i < 4 * SUB; ++i) {
          const bool keep = e[i] >= kh;
          if (keep && kept < C::CAPE)
            out[kept] = (int)((e[i] & 0xffff0000u) | (unord32(e[i]) & 0xffffu));
          kept += keep ? 1 : 0;
        }
        cand_cnt[(int64_t)p * S + s] = (flag || kept > C::CAPE) ? -1 : kept;
        cand_h[2 * ((int64_t)p * S + s)] = hc;       // this slice's final threshold
        cand_h[2 * ((int64_t)p * S + s) + 1] = epc;  // the query's error bound
      }
    }
    }  // column halves
    if (!final_pass) {
      dmlp::wave_sync();
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        addr[ct] = lim[ct] - (SUB - CHECK) * 16 + 16 * sbuf[(ct * 16 + c) * C::CP + 4 * SUB + kg];
      pull_h();
      if (MODE & 128) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) h[ct] = INFINITY;
      }
      // resolve these LDS loads here, not at the next use: otherwise the waitcnt pass sees them
      // pending after the conditional call and drains lgkmcnt at every following step
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    }
  };

  // ---- D-deep register ring of step fragments + double-buffered accumulators
  bf16x8 A[D][KT];
  f32x4 Xi[D];
  f32x4 acc[2][CT];
#define DMLP_LOADA(J, R)                                                                        \
  do {                                                                                          \
    if ((MODE & 32) && ((J) & 1)) break;                                                        \
    if ((MODE & 64) && ((J) & 3)) break;                                                        \
    _Pragma("unroll") for (int kt = 0; kt < KT; ++kt)                                           \
      A[R][kt] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(              \
          xr, lane * 16 + kt * ks, (J) * (KT * ks), 0));                                        \
  } while (0)
#define DMLP_LOADX(J, R)                                                                        \
  do {                                                                                          \
    if (!(MODE & 4))                                                                            \
      Xi[R] = *(__attribute__((address_space(3))) const f32x4*)(size_t)(                        \
          xrb + (((J) >> 2) & 1) * 256 + ((J) & 3) * 64 + kg * 16);                             \
  } while (0)
#define DMLP_LOAD(J, R)                                                                         \
  do {                                                                                          \
    DMLP_LOADA(J, R);                                                                           \
    DMLP_LOADX(J, R);                                                                           \
  } while (0)
  // ring: step R of the tile in LDS slot SL
#define DMLP_RLOAD(SL, R)                                                                       \
  do {                                                                                          \
    _Pragma("unroll") for (int kt = 0; kt < KT; ++kt)                                           \
      A[R][kt] = *(__attribute__((address_space(3))) const bf16x8*)(size_t)(                    \
          ringA + (SL) * C::TILEB + ((R) * KT + kt) * 1024 + lane * 16);                        \
    Xi[R] = *(__attribute__((address_space(3))) const f32x4*)(size_t)(                          \
        ringN + (SL) * 256 + (R) * 64 + kg * 16);                                               \
  } while (0)
#define DMLP_MFMA(R, AB)                                                                        \
  do {                                                                                          \
    _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                         \
      acc[AB][ct] = mfma16<F16>(A[R][0], bh[ct][0], (MODE & 4) ? f32x4{0, 0, 0, 0} : Xi[R]);      \
      _Pragma("unroll") for (int kt = 1; kt < KT; ++kt)                                         \
        acc[AB][ct] = mfma16<F16>(A[R][kt], bh[ct][kt], acc[AB][ct]);                           \
    }                                                                                           \
  } while (0)
#define DMLP_EPILOGUE(AB, J)                                                                    \
  do {                                                                                          \
    /* per column tile: the 4-row group max, and the wave's hit mask straight from the        \
       compare (an SGPR pair: the uniform branches below test it with one s_cmp) */            \
    float m_[CT];                                                                               \
    unsigned long long hm_[CT];                                                                 \
    unsigned long long any_ = 0;                                                                \
    _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                         \
      m_[ct] = fmaxf(fmaxf(acc[AB][ct][0], acc[AB][ct][1]), fmaxf(acc[AB][ct][2], acc[AB][ct][3])); \
      hm_[ct] = __builtin_amdgcn_ballot_w64(m_[ct] >= h[ct]);                                   \
      any_ |= hm_[ct];                                                                          \
    }                                                                                           \
    if (MODE & 8) {                                                                             \
      if (lane == 0) atomicAdd(&g_x1_dbg[0], 1ull);                                             \
    }                                                                                           \
    if (!(MODE & 1) && (C::D == 4 || (J) < nsteps) && any_) {                                   \
      if (MODE & 8) {                                                                           \
        int np_ = 0;                                                                            \
        _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) np_ += __popcll(hm_[ct]);             \
        if (lane == 0) { atomicAdd(&g_x1_dbg[1], 1ull);                                         \
                         atomicAdd(&g_x1_dbg[2], (unsigned long long)np_); }                    \
      }                                                                                         \
      unsigned gl_ = (unsigned)((J) * 4 + kg);                                                  \
      asm volatile("" : "+v"(gl_)); /* one VGPR: each key is a single v_and_or / v_bfi */       \
      if (MODE & 512) {                                                                         \
        /* per column tile, a wave-uniform branch on its own hit mask: a taken step pays the   \
           append VALU only for the tiles some lane hit (~2 lane-keys of 256 per taken step) */ \
        _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                     \
          if (hm_[ct]) {                                                                        \
            *(__attribute__((address_space(3))) unsigned*)(size_t)addr[ct] =                   \
                (__float_as_uint(m_[ct]) & 0xffff0000u) | gl_;                                  \
            addr[ct] += m_[ct] >= h[ct] ? 16u : 0u;                                             \
          }                                                                                     \
        }                                                                                       \
      } else if (MODE & 256) {                                                                  \
        /* per tile, only the lanes that hit (exec-masked) store and advance */                 \
        _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                     \
          if (m_[ct] >= h[ct]) {                                                                \
            *(__attribute__((address_space(3))) unsigned*)(size_t)addr[ct] =                   \
                (__float_as_uint(m_[ct]) & 0xffff0000u) | gl_;                                  \
            addr[ct] += 16u;                                                                    \
          }                                                                                     \
        }                                                                                       \
      } else {                                                                                  \
      /* branch-free: every lane writes its entry to the next free slot and advances only on  \
         a hit (slot cnt <= SUB-1 exists; a miss is overwritten later and never read) */     \
      _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                       \
        *(__attribute__((address_space(3))) unsigned*)(size_t)addr[ct] =                       \
            (__float_as_uint(m_[ct]) & 0xffff0000u) | gl_;                                      \
        addr[ct] += m_[ct] >= h[ct] ? 16u : 0u;                                                 \
        if (MODE & 1024) trig_acc |= __builtin_amdgcn_ballot_w64(addr[ct] > lim[ct]);           \
      }                                                                                         \
      }                                                                                         \
    }                                                                                           \
  } while (0)
  // one compaction call site per CHECK steps (each inlined copy is ~8 KiB of code: one per
  // step of the unrolled ring would not stay in the instruction cache).  Ring: a tile this wave
  // issued is published before the (long) compaction, so the other waves never wait on it.
#define DMLP_CHECK()                                                                            \
  do {                                                                                          \
    /* the fill test at the check point itself (addresses only grow between checks): one    \
       compare per column tile every CHECK steps instead of one per tile per taken step */   \
    unsigned long long trig = 0;                                                                \
    if (MODE & 1024) {                                                                          \
      trig = trig_acc;                                                                          \
      trig_acc = 0;                                                                             \
    } else {                                                                                    \
      _Pragma("unroll") for (int ct = 0; ct < CT; ++ct)                                         \
        trig |= __builtin_amdgcn_ballot_w64(addr[ct] > lim[ct]);                                \
    }                                                                                           \
    if (trig) {                                                                                 \
      if (RING && pend >= 0) {                                                                  \
        publish(pend);                                                                          \
        pend = -1;                                                                              \
      }                                                                                         \
      compact(false);                                                                           \
    }                                                                                           \
  } while (0)

  // EARLY START: a new slice's max norm raises the eps of every column (see above); the owners
  // update oe / oh, the MFMA layout takes the new thresholds by the shuffle
  auto grow = [&](float xm) {
#pragma unroll
    for (int hb = 0; hb < NH; ++hb) {
      const int p = pbase + lane + 64 * hb;
      if (p < nq) {
        const float e_new = eps_of(qn[qidx[p]], xm);
        if (oh[hb] > -FLT_MAX && oh[hb] < INFINITY) oh[hb] -= 2.0f * (e_new - oe[hb]);
        oe[hb] = e_new;
      }
    }
    if (MODE & 128) {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const float hn = __shfl(oh[ct >> 2], (ct & 3) * 16 + c);
        h[ct] = h[ct] == INFINITY ? h[ct] : hn;
      }
    } else {
      pull_h();
    }
  };
  auto fail_all = [&]() {  // the data never arrived: report overflow, stop appending
#pragma unroll
    for (int hb = 0; hb < NH; ++hb) {
      ofl[hb] = 1;
      oh[hb] = INFINITY;
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) h[ct] = INFINITY;
  };
  if (rdy && rdy_fail) {
    fail_all();
    have = rdy_n;
  }
  unsigned long long trig_acc = 0;  // MODE 1024 (ablation): the fill test per taken step
  if constexpr (RING > 0) {
    if (nsteps > 0) {
      // tile 0 into the register ring, then per tile i: publish / claim + issue tile i + L,
      // wait for tile i + 1, and run tile i's 4 steps while reading tile i + 1 out of LDS
#pragma unroll
      for (int r = 0; r < 4; ++r) DMLP_RLOAD(0, r);
      done_read(0);
      for (int i = 0; i < nt; ++i) {
        if (pend >= 0) {
          publish(pend);
          pend = -1;
        }
        const int sl1 = (i + 1) % RS;
        // both counter reads issue before step 0's MFMAs and are consumed after them (consuming
        // them two steps later, with tile i + 1's reads at steps 2 and 3, measured slower: r9x)
        const unsigned nx = __hip_atomic_load(rnext, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const unsigned rd = __hip_atomic_load(rready + sl1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int j = i * 4 + r;
          DMLP_MFMA(r, r & 1);
          if (r == 0) {
            if (i + L < nt && claim_v(i + L, (unsigned)__builtin_amdgcn_readfirstlane((int)nx))) {
              produce(i + L);
              pend = i + L;
            }
            if (i + 1 < nt) {
              if (!lds_wait_v(rready + sl1, (unsigned)((i + 1) / RS + 1),
                              (unsigned)__builtin_amdgcn_readfirstlane((int)rd)))
                ring_fail();
              if (rdy && have < rdy_n) {  // eps over tile i + 1's slice before any of it is judged
                const int si = min((i + 1) / rdy_tiles, rdy_n - 1);
                if (si >= have) {
                  const int need = widen(si);
                  const float xm = fold_xnm(xnmax, have, need);
                  have = need + 1;
                  if (xm > xnmax) {
                    grow(xm);
                    xnmax = xm;
                    ++n_grow;
                  }
                }
              }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          }
          DMLP_RLOAD(sl1, r);  // (past the last tile: a stale slot, never used)
          if (j > 0) DMLP_EPILOGUE((r + 1) & 1, j - 1);
          if (r % CHECK == CHECK - 1) DMLP_CHECK();
        }
        if (i + 1 < nt) done_read(i + 1);
      }
      DMLP_EPILOGUE(1, nsteps - 1);
      // a failed wait anywhere in the workgroup: every wave's queries report overflow
      if (lds_ld(rfail)) fail_all();
    }
  } else {
  // The C-operand ring: window w (steps 4w .. 4w + 3, 64 floats) sits in LDS slot w & 1; lane L
  // moves float L of a window (one dword per lane, 4 steps ahead of its first read).  16 lanes
  // read each 16-byte row group (an LDS broadcast), so the per-step norm traffic leaves the
  // texture path — which the fragment loads keep busy (profiles/r2b_screen_x1_ta_pmc.txt).
  static_assert(D == 4, "the C-operand ring assumes a 4-deep fragment ring");
  const unsigned xrb = C::LDS - C::XRING;  // LDS byte offset of the ring
  float xw = 0.0f;                          // the next window's float of this lane
  auto xwin = [&](int w) __attribute__((always_inline)) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ir, lane * 4, w * 256, 0));
  };
  if (nsteps > 0) {
    if (!(MODE & 4)) {
      *(__attribute__((address_space(3))) float*)(size_t)(xrb + lane * 4) = xwin(0);
      xw = xwin(1);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the ring reads stay after it
    }
    // prologue in the loop's issue order (A, Xi per step), so the waitcnt at the loop head is
    // the steady-state vmcnt(2 * (D - 1)), not a merge with a reordered prologue
#pragma unroll
    for (int r = 0; r < D; ++r) {
      DMLP_LOAD(r, r);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int j0 = 0; j0 < nsteps; j0 += D) {
      if (rdy && have < rdy_n) {
        // this iteration's loads reach tile (j0 + 11) / 4 (C-operand window j0/4 + 2)
        int need = min(((j0 + 11) >> 2) / rdy_tiles, rdy_n - 1);
        if (need >= have) {
          const int need1 = widen(need);
          bool ok = true;
          if (need1 == need)  // (all landed: no per-slice probes)
            for (int i = have; i <= need && ok; ++i) ok &= wait_slice(i);
          need = need1;
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope (host DMA)
          const int from = have;
          have = need + 1;
          if (ok) {
            const float xm = fold_xnm(xnmax, from, need);
            if (xm > xnmax) {
              grow(xm);
              xnmax = xm;
              ++n_grow;
            }
          } else {
            fail_all();
            have = rdy_n;
          }
        }
      }
#pragma unroll
      for (int r = 0; r < D; ++r) {
        const int j = j0 + r;  // D = 4: j < nsteps (nsteps % 4 == 0); D = 8: guarded epilogue
        DMLP_MFMA(r, r & 1);
        if (r == 0 && !(MODE & 4)) {
          // window j0/4 + 1 (steps j0 + 4 .. j0 + 7) into the slot window j0/4 - 1 used (every
          // read of it is done: those steps were loaded into the register ring already)
          *(__attribute__((address_space(3))) float*)(size_t)(
              xrb + (((j0 >> 2) + 1) & 1) * 256 + lane * 4) = xw;
          xw = xwin((j0 >> 2) + 2);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
        DMLP_LOAD(j + D, r);
        if (MODE & 2) {  // ablation: keep every MFMA result alive, no epilogue at all
          _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) asm volatile("" ::"v"(acc[r & 1][ct]));
        } else if (j > 0) {
          DMLP_EPILOGUE((r + 1) & 1, j - 1);
        }
        if (r % CHECK == CHECK - 1) DMLP_CHECK();
      }
    }
    // the last issued step (padded up to a multiple of D; the guard skips padding for D = 8)
    const int jl = ((nsteps + D - 1) / D) * D - 1;
    DMLP_EPILOGUE(jl & 1, jl);
  }
  }
#undef DMLP_LOAD
#undef DMLP_LOADA
#undef DMLP_LOADX
#undef DMLP_RLOAD
#undef DMLP_MFMA
#undef DMLP_EPILOGUE
#undef DMLP_CHECK
  if (MODE & 1) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) asm volatile("" ::"v"(acc[0][ct]), "v"(acc[1][ct]));
  }
  // final threshold over everything buffered, then the candidate ids
  compact(true);
  if (rdy && estats && lane == 0 && (n_wait | n_grow | n_to | n_qwait)) {
    atomicAdd(estats + 0, n_wait);
    atomicAdd(estats + 1, n_grow);
    atomicAdd(estats + 2, n_to);
    atomicAdd(estats + 3, n_qwait);
  }
}

int x1_sub(int kmax) { return kmax <= 16 ? 16 : 32; }

// column tiles per wave of the SUB = 16 (k <= 16) variants.  8 (128 queries per wave, one wave
// per SIMD) halves the vector-memory instructions per MFMA — the 4-tile kernel keeps the texture
// addresser ~75 % busy (TA_TA_BUSY, profiles/r2b_screen_x1_ta_pmc.txt) — but measured 2.39 ms
// against 1.38 ms on the bench shape: without a partner wave nothing covers the in-order epilogue.
// Kept as an A/B switch (DMLP_X1_CT=8).  SUB = 32 always uses 4.
int g_x1_ct = 4;
int x1_ct(int kmax) { return x1_sub(kmax) == 16 ? g_x1_ct : 4; }

// the LDS-ring variants (RING > 0): DMLP_X1_RING = 0 (off) or the sub-buffer depth of the ring
// kernel — 16 (5-tile ring), 14 (9 tiles) or 12 (13 tiles): a shallower candidate buffer leaves
// more LDS to the ring, i.e. more slack between the fastest and the slowest wave, at the price
// of more frequent compactions (and 40 / 48 instead of 56 kept group entries per column; 8-tile
// rings, a mask per slot index, measured slower: r9x)
int g_x1_ring = -1;
int64_t g_x1_ring_launches = 0;
int x1_ring() {
  if (g_x1_ring < 0) {
    const char* e = getenv("DMLP_X1_RING");
    const int v = e ? atoi(e) : 0;
    g_x1_ring = (v == 16 || v == 14 || v == 12) ? v : 0;
  }
  return g_x1_ring;
}
int x1_num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}
// the ring kernel fills the chip only with a workgroup (8 x 64 queries of a slice) per CU (tests
// force it onto smaller grids: g_x1_ring_force)
int g_x1_ring_force = 0;
bool x1_ring_fits(int nq, int S) {
  return x1_ring() && (g_x1_ring_force || (int64_t)((nq + 511) / 512) * S >= x1_num_cus());
}

template <int KT, int SUB, int DEPTH, int CHECK, int CTV, bool F16, int RING = 0>
int launch_x1(int hl, const void* xfrag, const float* xinit, int64_t n_tiles, int64_t n_points,
              const void* qhi, const float* qn, const int* qidx, const int* qk, int nq,
              const unsigned* xnmax, const unsigned* bad, float r1, float r2, float r3, int S,
              int* cand_ids, int* cand_cnt, float* cand_h, hipStream_t stream,
              const float* hseed = nullptr, int ccap = 0, const unsigned* rdy = nullptr,
              int rdy_tiles = 1, int rdy_n = 0, const unsigned* xnm_sl = nullptr,
              unsigned* estats = nullptr, long long rdy_to = 0,
              const unsigned* qrdy = nullptr, int qrdy_q = 1) {
  using C = X1Cfg<KT, SUB, DEPTH, CHECK, CTV, RING>;
  const int n_qblocks = ((nq + C::NCOL - 1) / C::NCOL + C::W - 1) / C::W;  // workgroups per slice
  const int tps = (int)((n_tiles + S - 1) / S);
  const int64_t grid = (int64_t)n_qblocks * S;
  if (grid <= 0) return 0;
  if constexpr (C::LDS > 65536) {  // past the default dynamic-LDS limit: raise it once
    static const hipError_t la = hipFuncSetAttribute(
        (const void*)k_screen_x1<KT, SUB, DEPTH, CHECK, CTV, 0, F16, RING>,
        hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    static const hipError_t lb = hipFuncSetAttribute(
        (const void*)k_screen_x1<KT, SUB, DEPTH, CHECK, CTV, 8, F16, RING>,
        hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (la != hipSuccess || lb != hipSuccess) return -(int)(la != hipSuccess ? la : lb);
  }
#define DMLP_X1_LAUNCH(M)                                                                      \
  hipLaunchKernelGGL((k_screen_x1<KT, SUB, DEPTH, CHECK, CTV, M, F16, RING>), dim3((unsigned)grid), dim3(C::W * 64), C::LDS, stream, \
                     (const u32x4*)xfrag, (const f32x4*)xinit, (int)n_tiles, (int)n_points,     \
                     (const bf16x8*)qhi, qn, qidx, qk, nq, xnmax, bad, r1, r2, r3, S, tps,      \
                     n_qblocks, hl, cand_ids, cand_cnt, cand_h, hseed, ccap, rdy, rdy_tiles,     \
                     rdy_n, xnm_sl, estats, rdy_to, qrdy, qrdy_q)
  if (hseed) {  // the COLLECT pass (SUB = 16, CT = 4, fp16 only: see dmlp_screen_x1_collect)
    if constexpr (SUB == 16 && CTV == 4 && F16 && RING == 0) DMLP_X1_LAUNCH(16);
    else return -3;
  } else if constexpr (RING > 0) {
    ++g_x1_ring_launches;
    if (x1_mode() == 8) DMLP_X1_LAUNCH(8);  // event counters
    else DMLP_X1_LAUNCH(0);
  } else if constexpr (KT <= 2) {
    // ablation modes only for the A <= 64 variants (each mode is a full kernel instantiation)
    switch (x1_mode()) {
      case 1: DMLP_X1_LAUNCH(1); break;
      case 2: DMLP_X1_LAUNCH(2); break;
      case 4: DMLP_X1_LAUNCH(4); break;
      case 6: DMLP_X1_LAUNCH(6); break;
      case 8: DMLP_X1_LAUNCH(8); break;
      case 32: DMLP_X1_LAUNCH(32); break;
      case 64: DMLP_X1_LAUNCH(64); break;
      case 128: DMLP_X1_LAUNCH(128); break;
      case 256: DMLP_X1_LAUNCH(256); break;
      case 512: DMLP_X1_LAUNCH(512); break;
      case 1024: DMLP_X1_LAUNCH(1024); break;

      default: DMLP_X1_LAUNCH(0); break;
    }
  } else {
    DMLP_X1_LAUNCH(0);
  }
#undef DMLP_X1_LAUNCH
  DMLP_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// Screen error bound of the single-term form, per query q (fp32 score a = <q',x'> - |x'|^2/2):
//   hi() = bf16(fp32(c)): |c - hi(c)| <= u|c|, u = 2^-9 (1 + 2^-15);  bf16 x bf16 products are
//   exact in fp32; the MFMA chain rounds at most A + 1 partial sums, each bounded by
//   sum|hi(q)hi(x)| + |x'|^2/2; xinit carries one fp32 rounding of |x'|^2/2.  With |x'| <= max:
//     |a - a_exact| <= r1 |q'| max|x'| + r2 max|x'|^2,
//     r1 = 2u + u^2 + (A+2) 2^-24 (1+u)^2,   r2 = (A+2) 2^-24 / 2 + 2^-24,
//   both taken x1.25 for the fp32 evaluation of the bound itself.
//
// fp16 operands (hl = 1): hi() = fp16(fp32(c)) has |c - hi(c)| <= u|c| + 2^-25 with
// u = 2^-11 (1 + 2^-12) (the 2^-25 is half an fp16 subnormal step: |c| < 2^-14), and
// fp16 x fp16 products are exact in fp32 as well, so the bound gains
//     r3 (sum_a |q_a| + |x_a|) <= r3 (|q'| + max|x'|),  r3 = 2^-25 (1 + u) sqrt(A),
// (x1.25 like the others) and the kernel adds r3 2^-15 >= A 2^-50 for the subnormal products.
extern "C" void dmlp_screen_x1_bound2(int A, int hl, float* r1, float* r2, float* r3) {
  const bool f16 = hl == 1;
  const double u = f16 ? std::ldexp(1.0, -11) * (1.0 + std::ldexp(1.0, -12))
                       : std::ldexp(1.0, -9) * (1.0 + std::ldexp(1.0, -15));
  const double e24 = std::ldexp(1.0, -24);
  *r1 = (float)(1.25 * (2.0 * u + u * u + (A + 2) * e24 * (1.0 + u) * (1.0 + u)));
  *r2 = (float)(1.25 * ((A + 2) * e24 * 0.5 + e24));
  *r3 = f16 ? (float)(1.25 * std::ldexp(1.0, -25) * (1.0 + u) * std::sqrt((double)A)) : 0.0f;
}
extern "C" void dmlp_screen_x1_bound(int A, float* r1, float* r2) {
  float r3;
  dmlp_screen_x1_bound2(A, 2, r1, r2, &r3);
}
// k <= 64 on one pass: the SUB = 32 buffers keep up to 120 group entries per column after a
// compaction (k + the 2 eps slack), and the group refine ranks up to 64 (KMAX) of <= 128 members
extern "C" int dmlp_screen_x1_kmax(void) { return 64; }
static bool x1_kt_ok(int KT) { return KT == 1 || KT == 2 || KT == 4 || KT == 8; }
extern "C" int dmlp_screen_x1_qw(int KT) { return x1_kt_ok(KT) ? 64 : 0; }
// queries per wave (= workgroup) of the variant that serves kmax
extern "C" int dmlp_screen_x1_cols(int KT, int kmax) {
  return x1_kt_ok(KT) ? 16 * (KT >= 4 ? 4 : x1_ct(kmax)) : 0;
}
// group ids per (query, slice) (refine expands each to its 4 members)
extern "C" int dmlp_screen_x1_cap(int kmax) { return 4 * (x1_sub(kmax) - 1); }
// resident workgroups (= waves) per CU: LDS-bound at 17.5 KiB (SUB 16, 4 tiles) / 33.5 KiB
// (SUB 32); the 8-tile variant runs one wave per SIMD (register-bound)
extern "C" int dmlp_screen_x1_waves_per_cu(int kmax) {
  return x1_sub(kmax) == 16 ? (x1_ct(kmax) == 8 ? 4 : 8) : 4;
}
// the same for an image of KT fragments per step: A > 64 (KT = 4, 8) runs one wave per SIMD (the
// query and ring fragments take the registers of two)
extern "C" int dmlp_screen_x1_waves_per_cu_kt(int KT, int kmax) {
  return KT >= 4 ? 4 : dmlp_screen_x1_waves_per_cu(kmax);
}
// a slice must stay below 2^16 4-row groups (16-bit group index in an entry)
extern "C" int64_t dmlp_screen_x1_min_slices(int64_t n_tiles) { return (n_tiles + 4095) / 4096; }
extern "C" void dmlp_set_x1_mode(int mode) { g_x1_mode = mode; }
// column tiles per wave of the k <= 16 variants (4 or 8; A/B)
extern "C" void dmlp_set_x1_ct(int ct) { g_x1_ct = ct == 4 ? 4 : 8; }
// the LDS-ring screen for k <= 16, A <= 32 (0 off; 16 / 14 / 12: its sub-buffer depth)
extern "C" void dmlp_set_x1_ring(int sub) { g_x1_ring = (sub == 16 || sub == 14 || sub == 12) ? sub : 0; }
extern "C" int dmlp_get_x1_ring(void) { return x1_ring(); }
// 1: the ring kernel whenever it is on, whatever the grid (tests); returns the previous value
extern "C" int dmlp_set_x1_ring_force(int on) {
  const int old = g_x1_ring_force;
  g_x1_ring_force = on ? 1 : 0;
  return old;
}
extern "C" int64_t dmlp_x1_ring_launches(void) { return g_x1_ring_launches; }
extern "C" int dmlp_x1_debug_counters(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x1_dbg), sizeof(g_x1_dbg));
  if (e != hipSuccess) return -(int)e;
  if (reset) {
    unsigned long long z[8] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_x1_dbg), z, sizeof(z));
    if (e != hipSuccess) return -(int)e;
  }
  return 0;
}

// ---- large k (32 < k <= 256) on the single-term screen, in two passes over the host's fp16
// operands: (1) dmlp_screen_x1 over S1 data slices with k' = ceil(k / S1) <= 16 per query (the
// cheap SUB = 16 variant) leaves each slice's final threshold h_s = a'_s - 2 eps (a'_s <= the
// k'-th best approximate score of the slice); since S1 k' >= k, the k-th best exact score over all
// slices is >= min_s (a'_s - eps), so hseed = min_s h_s keeps every true top-k member (any approx
// score >= exact - eps).  (2) dmlp_screen_x1_collect re-screens everything at that fixed threshold
// and flushes the passing 4-row groups to per-(query, slice) global lists; the group refine
// (dmlp_refine_groups2, collect = 1) takes the k-th largest group key over the lists.
__global__ __launch_bounds__(256) void k_x1_seed(const float* __restrict__ cand_h,
                                                 const int* __restrict__ cand_cnt, int S1, int nq,
                                                 float* __restrict__ hseed) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= nq) return;
  float m = INFINITY;
  bool bad = false;
  for (int s = 0; s < S1; ++s) {
    bad |= cand_cnt[(int64_t)p * S1 + s] < 0;  // overflowed: its threshold is lost
    m = fminf(m, cand_h[2 * ((int64_t)p * S1 + s)]);
  }
  hseed[p] = bad ? INFINITY : m;  // +inf: the COLLECT pass reports the query as overflowed
}

extern "C" int dmlp_x1_seed(const float* cand_h, const int* cand_cnt, int S1, int nq,
                            float* hseed, void* stream) {
  if (nq <= 0) return 0;
  if (S1 < 1) return -1;
  hipLaunchKernelGGL(k_x1_seed, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, cand_h, cand_cnt, S1, nq, hseed);
  DMLP_LAUNCH_CHECK();
  return 0;
}

// The COLLECT pass over the host's fp16 image (hl = 1): hseed[p] per query position p (+inf: the
// query reports overflow), ccap group ids per (query, slice); cand_cnt = -1 past ccap.
extern "C" int dmlp_screen_x1_collect(int KT, int A, const void* xfrag, const float* xinit,
                                      int64_t n_tiles, int64_t n_points, const void* qhi,
                                      const float* qn, const int* qidx, const int* qk, int nq,
                                      const unsigned* xnmax_bits, const unsigned* bad,
                                      const float* hseed, int ccap, int S, int* cand_ids,
                                      int* cand_cnt, float* cand_h, void* stream) {
  if (nq <= 0) return 0;
  if (!hseed || ccap < 1 || S < 1 || n_tiles < 0 || n_tiles > 0x7fffffff / 64 ||
      n_points > n_tiles * 64)
    return -1;
  if ((n_tiles + S - 1) / S > 4096) return -4;  // 16-bit group index per slice
  if (!x1_kt_ok(KT) || A > KT * 32) return -3;
  float r1, r2, r3;
  dmlp_screen_x1_bound2(A, 1, &r1, &r2, &r3);
  hipStream_t st = (hipStream_t)stream;
#define DMLP_X1C(KTV)                                                                           \
  return launch_x1<KTV, 16, 4, 2, 4, true>(1, xfrag, xinit, n_tiles, n_points, qhi, qn, qidx,   \
                                          qk, nq, xnmax_bits, bad, r1, r2, r3, S, cand_ids,    \
                                          cand_cnt, cand_h, st, hseed, ccap)
  if (KT == 1) DMLP_X1C(1);
  if (KT == 2) DMLP_X1C(2);
  if (KT == 4) DMLP_X1C(4);
  DMLP_X1C(8);
#undef DMLP_X1C
}

extern "C" int dmlp_screen_x1(int KT, int hl, int A, const void* xfrag, const float* xinit,
                              int64_t n_tiles, int64_t n_points, const void* qhi, const float* qn,
                              const int* qidx, const int* qk, int nq, int kmax,
                              const unsigned* xnmax_bits, const unsigned* bad, int S,
                              int* cand_ids, int* cand_cnt, float* cand_h, void* stream) {
  if (nq <= 0) return 0;
  if (S < 1 || n_tiles < 0 || n_tiles > 0x7fffffff / 64 || n_points > n_tiles * 64) return -1;
  if ((n_tiles + S - 1) / S > 4096) return -4;  // 16-bit group index per slice
  if (kmax > 64 || !x1_kt_ok(KT) || A > KT * 32) return -3;
  if (hl != 1 && hl != 2) return -1;
  float r1, r2, r3;
  dmlp_screen_x1_bound2(A, hl, &r1, &r2, &r3);
  hipStream_t st = (hipStream_t)stream;
#define DMLP_X1_ARGS hl, xfrag, xinit, n_tiles, n_points, qhi, qn, qidx, qk, nq, xnmax_bits, bad, r1, \
                     r2, r3, S, cand_ids, cand_cnt, cand_h, st
  const int sub = x1_sub(kmax);
  const int ct = x1_ct(kmax);
  // hl = 1: the host's fp16 image + fp16 query fragments; hl = 2: prep.hip's bf16 hi/lo image
#define DMLP_X1_PICK(F16)                                                                      \
  do {                                                                                         \
    if (KT == 1) {                                                                             \
      if (sub == 32) return launch_x1<1, 32, 4, 2, 4, F16>(DMLP_X1_ARGS);                      \
      if (ct == 4 && x1_ring_fits(nq, S)) {                                                    \
        if (x1_ring() == 16) return launch_x1<1, 16, 4, 2, 4, F16, 5>(DMLP_X1_ARGS);           \
        if (x1_ring() == 14) return launch_x1<1, 14, 4, 2, 4, F16, 9>(DMLP_X1_ARGS);           \
        return launch_x1<1, 12, 4, 2, 4, F16, 13>(DMLP_X1_ARGS);                               \
      }                                                                                        \
      return ct == 8 ? launch_x1<1, 16, 4, 2, 8, F16>(DMLP_X1_ARGS)                            \
                     : launch_x1<1, 16, 4, 2, 4, F16>(DMLP_X1_ARGS);                           \
    }                                                                                          \
    if (KT == 2) {                                                                             \
      if (sub == 32) return launch_x1<2, 32, 4, 2, 4, F16>(DMLP_X1_ARGS);                      \
      return ct == 8 ? launch_x1<2, 16, 4, 2, 8, F16>(DMLP_X1_ARGS)                            \
                     : launch_x1<2, 16, 4, 2, 4, F16>(DMLP_X1_ARGS);                           \
    }                                                                                          \
    if (KT == 4) {                                                                             \
      if (sub == 32) return launch_x1<4, 32, 4, 2, 4, F16>(DMLP_X1_ARGS);                      \
      return launch_x1<4, 16, 4, 2, 4, F16>(DMLP_X1_ARGS);                                     \
    }                                                                                          \
    if (sub == 32) return launch_x1<8, 32, 4, 2, 4, F16>(DMLP_X1_ARGS);                        \
    return launch_x1<8, 16, 4, 2, 4, F16>(DMLP_X1_ARGS);                                       \
  } while (0)
  if (hl == 1) DMLP_X1_PICK(true);
  DMLP_X1_PICK(false);
#undef DMLP_X1_PICK
#undef DMLP_X1_ARGS
}

// The single-term screen over the host's fp16 image while that image is still crossing PCIe
// (fast_step.hip's early start): one data slice per workgroup (S = 1), rdy[i] != 0 once image
// tiles [i rdy_tiles, (i + 1) rdy_tiles) and their max norm xnm_sl[i] (fp32 bits) landed.  The
// result is the one dmlp_screen_x1(KT, 1, ...) gives with S = 1 once every slice landed.
// ... with the query operands in flight too (qrdy != null): qrdy[b] != 0 once queries
// [b qrdy_q, (b + 1) qrdy_q) have their fragments and norms on the device (qrdy_q a multiple of
// 128, a wave's columns); the waits for them are counted into estats[3].
extern "C" int dmlp_screen_x1_early2(int KT, int A, const void* xfrag, const float* xinit,
                                     int64_t n_tiles, int64_t n_points, const void* qhi,
                                     const float* qn, const int* qidx, const int* qk, int nq,
                                     int kmax, const unsigned* bad, const unsigned* rdy,
                                     int rdy_tiles, int rdy_n, const unsigned* xnm_sl,
                                     int* cand_ids, int* cand_cnt, float* cand_h,
                                     unsigned* estats, const unsigned* qrdy, int qrdy_q,
                                     void* stream);
extern "C" int dmlp_screen_x1_early(int KT, int A, const void* xfrag, const float* xinit,
                                    int64_t n_tiles, int64_t n_points, const void* qhi,
                                    const float* qn, const int* qidx, const int* qk, int nq,
                                    int kmax, const unsigned* bad, const unsigned* rdy,
                                    int rdy_tiles, int rdy_n, const unsigned* xnm_sl,
                                    int* cand_ids, int* cand_cnt, float* cand_h,
                                    unsigned* estats, void* stream) {
  return dmlp_screen_x1_early2(KT, A, xfrag, xinit, n_tiles, n_points, qhi, qn, qidx, qk, nq, kmax,
                               bad, rdy, rdy_tiles, rdy_n, xnm_sl, cand_ids, cand_cnt, cand_h,
                               estats, nullptr, 128, stream);
}
extern "C" int dmlp_screen_x1_early2(int KT, int A, const void* xfrag, const float* xinit,
                                     int64_t n_tiles, int64_t n_points, const void* qhi,
                                     const float* qn, const int* qidx, const int* qk, int nq,
                                     int kmax, const unsigned* bad, const unsigned* rdy,
                                     int rdy_tiles, int rdy_n, const unsigned* xnm_sl,
                                     int* cand_ids, int* cand_cnt, float* cand_h,
                                     unsigned* estats, const unsigned* qrdy, int qrdy_q,
                                     void* stream) {
  if (nq <= 0) return 0;
  if (n_tiles < 1 || n_tiles > 4096 || n_points > n_tiles * 64 || !rdy || !xnm_sl ||
      rdy_tiles < 1 || rdy_n < 1 || (int64_t)rdy_tiles * rdy_n < n_tiles)
    return -1;
  // (qrdy: the list must be every query in order, qidx[p] == p — the all-queries pass)
  if (qrdy && (qrdy_q < 128 || qrdy_q % 128 != 0)) return -1;
  if (kmax > 64 || !x1_kt_ok(KT) || A > KT * 32) return -3;
  float r1, r2, r3;
  dmlp_screen_x1_bound2(A, 1, &r1, &r2, &r3);
  hipStream_t st = (hipStream_t)stream;
  const int sub = x1_sub(kmax), ct = x1_ct(kmax);
  // the wait bound: DMLP_EARLY_TIMEOUT_MS (default 50) of the constant-rate wall clock
  static const long long rdy_to = [] {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
      khz = 100000;  // 100 MHz
    const char* e = getenv("DMLP_EARLY_TIMEOUT_MS");
    const double ms = e ? atof(e) : 50.0;
    return (long long)(ms * khz);
  }();
#define DMLP_X1E(KTV, SUBV, CTV, ...)                                                           \
  return launch_x1<KTV, SUBV, 4, 2, CTV, true, ##__VA_ARGS__>(1, xfrag, xinit, n_tiles, n_points, qhi, qn, qidx, \
                                               qk, nq, bad, bad, r1, r2, r3, 1, cand_ids,      \
                                               cand_cnt, cand_h, st, nullptr, 0, rdy, rdy_tiles, \
                                               rdy_n, xnm_sl, estats, rdy_to, qrdy, qrdy_q)
  if (KT == 1) {
    if (sub == 32) DMLP_X1E(1, 32, 4);
    if (ct == 8) DMLP_X1E(1, 16, 8);
    if (x1_ring_fits(nq, 1)) {
      if (x1_ring() == 16) DMLP_X1E(1, 16, 4, 5);
      if (x1_ring() == 14) DMLP_X1E(1, 14, 4, 9);
      DMLP_X1E(1, 12, 4, 13);
    }
    DMLP_X1E(1, 16, 4);
  }
  if (KT == 2) {
    if (sub == 32) DMLP_X1E(2, 32, 4);
    if (ct == 8) DMLP_X1E(2, 16, 8);
    DMLP_X1E(2, 16, 4);
  }
  if (KT == 4) {
    if (sub == 32) DMLP_X1E(4, 32, 4);
    DMLP_X1E(4, 16, 4);
  }
  if (sub == 32) DMLP_X1E(8, 32, 4);
  DMLP_X1E(8, 16, 4);
#undef DMLP_X1E
}
