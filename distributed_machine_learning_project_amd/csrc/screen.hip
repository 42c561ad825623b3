// screen.hip — the fused hot kernel: bf16x3 MFMA distance screen + streaming per-query
// threshold + candidate compaction (SURVEY.md §2.5 K2+K3, §7.4 H1/H2).
//
// Reference hot loop: for every (query, point) an exact fp64 distance and a heap/nth_element
// top-k (engine.cpp:235-256; bench_1 @0xcf38-0xd10c; bench_4 @0xcb80).  Exact fp64 costs
// 3 fp64 VALU ops per (pair, attribute); this kernel instead computes a SCORE
//     a(q,x) = <q-mu, x-mu> - |x-mu|^2 / 2   ( = (|q-mu|^2 - d(q,x)) / 2 )
// on the matrix cores with a 3-term bf16 split (hi*hi + hi*lo + lo*hi, fp32 accumulate;
// mfma_f32_16x16x32_bf16), then keeps, per query, every point whose score could still belong
// to the exact top-k.  With |a - a_exact| <= eps_q (rigorous bound, see ops/knn.py) and a_k the
// k-th largest score buffered so far, every point with a < a_k - 2*eps_q is provably outside
// the exact top-k (and not even tied), so the per-query threshold h = a_k - 2*eps_q only rises.
// Survivors are re-ranked exactly (fp64, no FMA, reference order) by refine.hip, so the final
// neighbour lists and checksums are bit-identical to the reference.
//
// Geometry (gfx950): one workgroup = WAVES waves, each wave owns 16 queries (one MFMA column
// tile) for the whole stream; query bf16 fragments live in VGPRs.  The data slice streams
// through a 2-deep LDS ring of 64-point tiles (lane-linear 1 KiB fragments laid out by
// prep.hip); a tile wider than KT = 4 (A in (128, 256]) streams as NST = KT / 4 stages of four
// 32-attribute fragments each (32 KiB + the norm row), the accumulators carried across a tile's
// stages and the epilogue run after its last one, so the ring stays 2 x 32 KiB.  Staging goes through registers (global_load_dwordx4 issued one step ahead,
// ds_write_b128 after the barrier): no LDS-DMA is ever in flight, so hipcc never has to drain
// vmcnt in front of the candidate-buffer LDS traffic.  Candidate buffers ({score, id} x CAP per
// query) live in LDS; append offsets come from in-register per-column counts and a 4-lane
// prefix (no LDS atomics).  When a buffer passes CAP-64 entries the owning wave compacts it
// alone (bitonic sort of the scores across the wave).
// Block -> (query block, data slice) is XCD-aware when S % 8 == 0: every XCD streams only its
// own S/8 slices, so each slice is fetched into exactly one XCD's L2.
//
// HL = 1: the single-term form on the host's fp16 image and fp16 query fragments (the operands
// screen_x1.hip reads, already on the device when the host rendered them): one
// v_mfma_f32_16x16x32_f16 per fragment instead of three bf16 products, half the LDS staging, and
// the single-term error bound (dmlp_screen_x1_bound2, ~2^-10 relative instead of ~2^-16: a few
// percent more candidates at k in (32, 256]).  Per-point (score, id) entries as for HL = 2.
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// Ablation switch for profiling only (bit 0: no candidate path, bit 1: no MFMA, bit 2: no tile
// streaming).  Results are wrong unless it is 0; set through dmlp_set_screen_mode.
int g_screen_mode = 0;
// mode & 8: event counters (steps, candidate-path entries, appended entries, compactions)
__device__ unsigned long long g_screen_dbg[8];
#define DMLP_DBG(I, V)                                      \
  do {                                                      \
    if (mode & 8) {                                         \
      const unsigned long long v_ = (V);                    \
      if (lane == 0) atomicAdd(&g_screen_dbg[(I)], v_);     \
    }                                                       \
  } while (0)

template <int KT, int WAVES, int CAP, int HL = 2>
struct ScreenCfg {
  static constexpr int KTS = KT > 4 ? 4 : KT;  // 32-attribute fragments per LDS stage
  static constexpr int NST = KT / KTS;         // stages per 64-point tile
  static constexpr int TILE_FRAGS = 4 * KT * HL;  // 1 KiB fragments per tile of the image
  static constexpr int FRAGS = 4 * KTS * HL;   // 1 KiB fragments per stage
  static constexpr int TILE_BYTES = FRAGS * 1024 + 256;
  static constexpr int G = FRAGS / WAVES;   // staged 16-B vectors per lane per tile
  static constexpr int D0 = G <= 2 ? 4 : (G <= 4 ? 3 : 2);
  static constexpr int D = (D0 + NST - 1) / NST * NST;  // register-ring depth (stages)
  static constexpr int SUB = CAP / 4;      // per-lane sub-buffer entries
  static constexpr int LDS = 2 * TILE_BYTES + WAVES * 64 * (SUB + 1) * 8;
  static_assert(FRAGS % WAVES == 0, "fragments must split evenly over waves");
  static_assert(KT % KTS == 0 && D % NST == 0, "a tile's stages must map to fixed ring slots");
  static_assert(LDS <= 163840, "LDS budget");
  static_assert(CAP % 64 == 0, "CAP multiple of 64");
};

template <int KT, int WAVES, int CAP, int HL>
__global__ __launch_bounds__(WAVES * 64, 1) void k_screen(
    const u32x4* __restrict__ xfrag, const float* __restrict__ xinit, int n_tiles,
    const bf16x8* __restrict__ qhi, const bf16x8* __restrict__ qlo, const float* __restrict__ qn,
    const int* __restrict__ qidx, const int* __restrict__ qk, int nq,
    const unsigned* __restrict__ xnmax_bits, const unsigned* __restrict__ bad, float eps_rel,
    float r1, float r2, float r3, int S, int tiles_per_slice, int n_qblocks, int mode,
    int* __restrict__ cand_ids, int* __restrict__ cand_cnt) {
  using C = ScreenCfg<KT, WAVES, CAP, HL>;
  constexpr int E = CAP / 64;
  constexpr int KTS = C::KTS, NST = C::NST;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const tiles = smem;
  i32x2* const bufs = (i32x2*)(smem + 2 * C::TILE_BYTES);
  constexpr int SUB = C::SUB;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c = lane & 15;   // MFMA column = query of this lane
  const int kg = lane >> 4;  // k-group / row group

  // ---- block -> (query block, slice), XCD-aware when S % 8 == 0
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
  const int nst = nt * NST;  // LDS stages of the slice

  // ---- this lane's query (column)
  const int pbase = (qb * WAVES + wave) * 16;
  const int p = pbase + c;
  const bool valid = p < nq;
  if (*bad) {  // data/queries outside the screen's range: every query takes the exact path
    if (valid && lane < 16) cand_cnt[(int64_t)p * S + s] = -1;
    return;
  }
  const float xnmax = __uint_as_float(*xnmax_bits);
  const int q = valid ? qidx[p] : 0;
  bf16x8 bh[KT], bl[HL == 2 ? KT : 1];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    bh[kt] = qhi[(q * KT + kt) * 4 + kg];
    if constexpr (HL == 2) bl[kt] = qlo[(q * KT + kt) * 4 + kg];
  }
  // |a - a_exact| <= eps: the 3-term bound (HL = 2), or screen_x1.hip's single-term fp16 bound
  const float eps = HL == 2 ? eps_rel * (qn[q] + xnmax)
                            : r1 * sqrtf(qn[q]) * sqrtf(xnmax) + r2 * xnmax +
                                  r3 * (sqrtf(qn[q]) + sqrtf(xnmax)) + r3 * 0x1p-15f;
  const int kq = valid ? qk[q] : 0;
  float h = valid ? -FLT_MAX : INFINITY;
  int cnt = 0;  // entries in this lane's own sub-buffer (negative: column overflowed)
  i32x2* const wbuf = bufs + wave * 64 * (SUB + 1);

  // ---- D-deep register ring for the stage stream: stage j lives in register set j % D, so D-1
  // stages are in flight while one is consumed (the stream is latency-bound otherwise).
  // Macros, not lambdas, and native vector types: HIP's uint4 (a union struct) and captured
  // arrays both defeat SROA and end up in scratch.
  constexpr int D = C::D;
  u32x4 stg[D][C::G];
  float stx[D];
  // Loads are issued unconditionally (stage index clamped, every wave fetches the 256-B xinit
  // row) so the vmcnt bookkeeping is path-independent and hipcc emits counted waits.  Stage
  // fragment f = (rt * KTS + ktl) * HL + hilo is image fragment (rt * KT + h * KTS + ktl) * HL +
  // hilo of its tile (h: the stage within the tile; the identity when NST = 1).
#define DMLP_LOAD_TILE(I, R)                                                      \
  do {                                                                            \
    const int i_ = (I) < nst ? (I) : nst - 1;                                     \
    const int t_ = t0 + i_ / NST, h_ = i_ % NST;                                  \
    const u32x4* src_ = xfrag + (int64_t)t_ * (C::TILE_FRAGS * 64);               \
    _Pragma("unroll") for (int g = 0; g < C::G; ++g) {                            \
      const int f_ = wave + g * WAVES, rt_ = f_ / (HL * KTS);                     \
      stg[R][g] = src_[((rt_ * KT + h_ * KTS) * HL + f_ - rt_ * HL * KTS) * 64 + lane]; \
    }                                                                             \
    stx[R] = xinit[(int64_t)t_ * 64 + lane];                                      \
  } while (0)
#define DMLP_STORE_TILE(I, R)                                                     \
  do {                                                                            \
    char* dst_ = tiles + ((I) & 1) * C::TILE_BYTES;                               \
    _Pragma("unroll") for (int g = 0; g < C::G; ++g)                              \
        *(u32x4*)(dst_ + (wave + g * WAVES) * 1024 + lane * 16) = stg[R][g];      \
    if (wave == 0) ((float*)(dst_ + C::FRAGS * 1024))[lane] = stx[R];             \
  } while (0)

  // ---- candidate buffers: column c owns 4 sub-buffers of SUB entries, one per row-group lane
  // (kg), so a lane appends to its own sub-buffer with no cross-lane coordination.  Each lane
  // appends at most 16 entries per tile; a column is compacted once any of its lanes holds more
  // than SUB-16 (its entries are then re-dealt round-robin over the 4 sub-buffers).
  i32x2* const wsub = wbuf;
  auto sub_ptr = [&](int cc, int m) { return wsub + (cc * 4 + m) * (SUB + 1); };

  // gather column cc's entries (E per lane, element idx = r*64 + lane) into registers
#define DMLP_GATHER(CC, EV, VALID, NTOT)                                                       \
  const int c0_ = __shfl(cnt, (CC)), c1_ = __shfl(cnt, (CC) + 16), c2_ = __shfl(cnt, (CC) + 32), \
            c3_ = __shfl(cnt, (CC) + 48);                                                      \
  const int NTOT = c0_ + c1_ + c2_ + c3_;                                                      \
  i32x2 EV[E];                                                                                 \
  bool VALID[E];                                                                               \
  _Pragma("unroll") for (int r = 0; r < E; ++r) {                                              \
    const int idx_ = r * 64 + lane;                                                            \
    const int m_ = idx_ / SUB, j_ = idx_ - m_ * SUB;                                           \
    const int cm_ = m_ == 0 ? c0_ : (m_ == 1 ? c1_ : (m_ == 2 ? c2_ : c3_));                   \
    VALID[r] = j_ < cm_;                                                                       \
    EV[r] = VALID[r] ? sub_ptr((CC), m_)[j_] : (i32x2){__float_as_int(-INFINITY), -1};         \
  }

  auto compact = [&](int cc) {
    DMLP_GATHER(cc, e, ok, ntot)
    const int kc = __shfl(kq, cc);
    DMLP_DBG(3, 1);
    if (ntot >= kc) {
      // k-th largest score by a 32-step radix descent over order-preserving keys (ballots only)
      unsigned u[E];
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const unsigned bits = (unsigned)e[r].x;
        u[r] = ok[r] ? (bits ^ ((bits >> 31) ? 0xffffffffu : 0x80000000u)) : 0u;
      }
      unsigned T = 0;
      // stopping at bit 12 leaves T <= the exact k-th key (low bits zero), i.e. a valid but
      // ~2^-11-relative-looser threshold; 20 ballot rounds instead of 32
      for (int bit = 31; bit >= 12; --bit) {
        const unsigned cand = T | (1u << bit);
        int cntge = 0;
#pragma unroll
        for (int r = 0; r < E; ++r) cntge += __popcll(__ballot(u[r] >= cand));
        if (cntge >= kc) T = cand;
      }
      const unsigned tb = (T >> 31) ? (T ^ 0x80000000u) : ~T;
      const float ak = __uint_as_float(tb);
      const float hn = ak - 2.0f * __shfl(eps, cc);
      if (c == cc) h = fmaxf(h, hn);
    }
    const float hc = __shfl(h, cc);
    int base = 0;
    dmlp::wave_sync();
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const bool keep = ok[r] && __int_as_float(e[r].x) >= hc;
      const unsigned long long m = __ballot(keep);
      if (keep) {
        const int pos = base + __popcll(m & dmlp::lanemask_lt());
        sub_ptr(cc, pos & 3)[pos >> 2] = e[r];
      }
      base += __popcll(m);
    }
    dmlp::wave_sync();
    if (c == cc) cnt = (base + 3 - kg) >> 2;
    if (base > CAP - 64) {  // pathological ties: give up on this query, exact fallback
      if (c == cc) { h = INFINITY; cnt = -(1 << 28); }
    }
  };

  // ---- prologue
  f32x4 acc[4];  // carried across the stages of a tile
  if (nst > 0) {
    DMLP_LOAD_TILE(0, 0);
    DMLP_STORE_TILE(0, 0);
#pragma unroll
    for (int r = 1; r < D; ++r) DMLP_LOAD_TILE(r, r);
  }

  for (int i0 = 0; i0 < nst; i0 += D) {
#pragma unroll
  for (int r = 0; r < D; ++r) {
    const int i = i0 + r;
    if (i >= nst) break;
    const int hs = r % NST;  // stage within the tile (i0 is a multiple of D, D of NST)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // set r held tile i (already in LDS): refill it with tile i+D.  Tile i+1 (set r+1) goes to
    // the other LDS buffer after this step's MFMAs; everyone finished reading that buffer at
    // step i-1, before the barrier above.
    if (!(mode & 4)) DMLP_LOAD_TILE(i + D, r);

    const char* tb = tiles + (i & 1) * C::TILE_BYTES;
    bf16x8 ah[4][KTS], al[4][HL == 2 ? KTS : 1];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      if (hs == 0) acc[rt] = *(const f32x4*)(tb + C::FRAGS * 1024 + rt * 64 + kg * 16);
#pragma unroll
      for (int kt = 0; kt < KTS; ++kt) {
        ah[rt][kt] = *(const bf16x8*)(tb + ((rt * KTS + kt) * HL + 0) * 1024 + lane * 16);
        if constexpr (HL == 2)
          al[rt][kt] = *(const bf16x8*)(tb + ((rt * KTS + kt) * 2 + 1) * 1024 + lane * 16);
      }
    }
#pragma unroll
    for (int kt = 0; kt < KTS; ++kt) {
      if (mode & 2) break;  // ablation: no matrix work
      const bf16x8 qh = bh[hs * KTS + kt];
      if constexpr (HL == 1) {  // single term: hi(q') * hi(x'), fp16 operands
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ah[rt][kt]),
                                                           __builtin_bit_cast(f16x8, qh), acc[rt],
                                                           0, 0, 0);
      } else {
        const bf16x8 ql = bl[hs * KTS + kt];
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[rt][kt], qh, acc[rt], 0, 0, 0);
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[rt][kt], ql, acc[rt], 0, 0, 0);
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[rt][kt], qh, acc[rt], 0, 0, 0);
      }
    }
    if (hs == NST - 1) {  // a whole tile accumulated: the epilogue
    float mr[4];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
      mr[rt] = fmaxf(fmaxf(acc[rt][0], acc[rt][1]), fmaxf(acc[rt][2], acc[rt][3]));
    const float mx = fmaxf(fmaxf(mr[0], mr[1]), fmaxf(mr[2], mr[3]));
    DMLP_DBG(0, 1);
    if ((mode & 1) == 0 && __ballot(mx >= h)) {
      DMLP_DBG(1, 1);
      if (mode & 8) {
        int np = 0;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int j = 0; j < 4; ++j) np += acc[rt][j] >= h ? 1 : 0;
        for (int off = 32; off > 0; off >>= 1) np += __shfl_xor(np, off);
        DMLP_DBG(2, np);
      }
      // candidate path: append this lane's passing (score, id) pairs to its own sub-buffer
      i32x2* mys = sub_ptr(c, kg);
      const int idbase = (t0 + i / NST) * 64 + kg * 4;
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
        if (__ballot(mr[rt] >= h)) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (acc[rt][j] >= h) {
              mys[cnt] = (i32x2){__float_as_int(acc[rt][j]), idbase + rt * 16 + j};
              ++cnt;
            }
          }
        }
      }
      unsigned long long nm = __ballot(cnt > SUB - 16);
      unsigned cols = (unsigned)((nm | (nm >> 16) | (nm >> 32) | (nm >> 48)) & 0xffffull);
      while (cols) {
        const int cc = __ffs(cols) - 1;
        cols &= cols - 1;
        compact(cc);
      }
    }
    if (mode & 1) asm volatile("" ::"v"(mx));  // keep the epilogue alive in ablations
    }  // epilogue
    if (!(mode & 4)) DMLP_STORE_TILE(i + 1, (r + 1) % D);  // past the end: idle buffer
  }
  }
#undef DMLP_LOAD_TILE
#undef DMLP_STORE_TILE

  // ---- write this slice's candidates (ids only; refine recomputes exact distances)
  dmlp::wave_sync();
  for (int cc = 0; cc < 16; ++cc) {
    const int pp = pbase + cc;
    if (pp >= nq) break;
    int* out = cand_ids + ((int64_t)pp * S + s) * CAP;
    if (__shfl(cnt, cc) < 0) {
      if (lane == 0) cand_cnt[(int64_t)pp * S + s] = -1;
      continue;
    }
    DMLP_GATHER(cc, e, ok, ntot)
    (void)ntot;
    const float hc = __shfl(h, cc);
    int base = 0;
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const bool keep = ok[r] && __int_as_float(e[r].x) >= hc;
      const unsigned long long m = __ballot(keep);
      if (keep) out[base + __popcll(m & dmlp::lanemask_lt())] = e[r].y;
      base += __popcll(m);
    }
    if (lane == 0) cand_cnt[(int64_t)pp * S + s] = base;
  }
#undef DMLP_GATHER
}

template <int KT, int WAVES, int CAP, int HL>
int launch_screen(const void* xfrag, const float* xinit, int64_t n_tiles, const void* qhi,
                  const void* qlo, const float* qn, const int* qidx, const int* qk, int nq,
                  const unsigned* xnmax, const unsigned* bad, float eps_rel, float r1, float r2,
                  float r3, int S, int* cand_ids, int* cand_cnt, hipStream_t stream) {
  using C = ScreenCfg<KT, WAVES, CAP, HL>;
  auto kern = k_screen<KT, WAVES, CAP, HL>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return -(int)e;
    attr_set = true;
  }
  const int n_qblocks = (nq + WAVES * 16 - 1) / (WAVES * 16);
  const int tps = (int)((n_tiles + S - 1) / S);
  const int64_t grid = (int64_t)n_qblocks * S;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WAVES * 64), C::LDS, stream,
                     (const u32x4*)xfrag, xinit, (int)n_tiles, (const bf16x8*)qhi,
                     (const bf16x8*)qlo, qn, qidx, qk, nq, xnmax, bad, eps_rel, r1, r2, r3, S, tps,
                     n_qblocks, g_screen_mode, cand_ids, cand_cnt);
  DMLP_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// (KT, CAP) -> WAVES, 3-term (HL = 2): LDS = 2*(8 KiB*min(KT, 4) + 256) + WAVES*16*CAP*8 <= 160 KiB
// (KT = 8: two 32 KiB stages per tile).  CAP = 512 serves 128 < k <= 256 (a column compacts to
// >= k entries and refills 448 - k before the next batch).
#define DMLP_SCREEN_CONFIGS(X)                                                                \
  X(1, 128, 8, 2) X(2, 128, 4, 2) X(3, 128, 4, 2) X(4, 128, 4, 2) X(1, 256, 4, 2)              \
  X(2, 256, 2, 2) X(3, 256, 2, 2) X(4, 256, 2, 2) X(1, 512, 2, 2) X(2, 512, 1, 2)              \
  X(3, 512, 1, 2) X(4, 512, 1, 2) X(8, 128, 4, 2) X(8, 256, 2, 2) X(8, 512, 1, 2)              \
  DMLP_SCREEN_CONFIGS_1(X)
// single-term fp16 (HL = 1, host image): half the staging, WAVES <= fragments per stage
#define DMLP_SCREEN_CONFIGS_1(X)                                                              \
  X(1, 128, 4, 1) X(2, 128, 8, 1) X(4, 128, 4, 1) X(8, 128, 4, 1) X(1, 256, 4, 1)              \
  X(2, 256, 4, 1) X(4, 256, 2, 1) X(8, 256, 2, 1) X(1, 512, 2, 1) X(2, 512, 2, 1)              \
  X(4, 512, 1, 1) X(8, 512, 1, 1)

extern "C" int dmlp_screen_kmax(int cap) {
  return cap == 128 ? 32 : (cap == 256 ? 128 : (cap == 512 ? 256 : 0));
}

extern "C" int dmlp_screen_lds_bytes_hl(int KT, int cap, int hl) {
#define DMLP_LDS_CASE(kt, cp, w, h) \
  if (KT == kt && cap == cp && hl == h) return ScreenCfg<kt, w, cp, h>::LDS;
  DMLP_SCREEN_CONFIGS(DMLP_LDS_CASE)
#undef DMLP_LDS_CASE
  return -1;
}
extern "C" int dmlp_screen_lds_bytes(int KT, int cap) { return dmlp_screen_lds_bytes_hl(KT, cap, 2); }

// waves per workgroup of the (KT, cap, hl) variant (-1: none)
extern "C" int dmlp_screen_waves_hl(int KT, int cap, int hl) {
#define DMLP_W_CASE(kt, cp, w, h) \
  if (KT == kt && cap == cp && hl == h) return w;
  DMLP_SCREEN_CONFIGS(DMLP_W_CASE)
#undef DMLP_W_CASE
  return -1;
}
extern "C" int dmlp_screen_waves(int KT, int cap) { return dmlp_screen_waves_hl(KT, cap, 2); }

// hl = 2: the 3-term screen on prep.hip's bf16 hi/lo image and device query fragments (qlo used,
// eps_rel the 3-term bound); hl = 1: the single-term screen on the host's fp16 image and fp16
// query fragments (qlo and eps_rel unused; A selects the single-term bound).
extern "C" int dmlp_screen_hl(int KT, int cap, int hl, int A, const void* xfrag,
                              const float* xinit, int64_t n_tiles, const void* qhi,
                              const void* qlo, const float* qn, const int* qidx, const int* qk,
                              int nq, const unsigned* xnmax_bits, const unsigned* bad,
                              float eps_rel, int S, int* cand_ids, int* cand_cnt, void* stream) {
  if (nq <= 0) return 0;
  if (S < 1 || n_tiles < 0 || n_tiles > 0x7fffffff / 64) return -1;
  if (hl != 1 && hl != 2) return -1;
  float r1 = 0.0f, r2 = 0.0f, r3 = 0.0f;
  if (hl == 1) {
    if (A < 1 || A > KT * 32) return -1;
    dmlp_screen_x1_bound2(A, 1, &r1, &r2, &r3);
  }
  hipStream_t st = (hipStream_t)stream;
#define DMLP_SCREEN_CASE(kt, cp, w, h)                                                          \
  if (KT == kt && cap == cp && hl == h)                                                         \
    return launch_screen<kt, w, cp, h>(xfrag, xinit, n_tiles, qhi, qlo, qn, qidx, qk, nq,       \
                                       xnmax_bits, bad, eps_rel, r1, r2, r3, S, cand_ids,       \
                                       cand_cnt, st);
  DMLP_SCREEN_CONFIGS(DMLP_SCREEN_CASE)
#undef DMLP_SCREEN_CASE
  return -2;
}

extern "C" int dmlp_screen(int KT, int cap, const void* xfrag, const float* xinit, int64_t n_tiles,
                           const void* qhi, const void* qlo, const float* qn, const int* qidx,
                           const int* qk, int nq, const unsigned* xnmax_bits, const unsigned* bad,
                           float eps_rel, int S, int* cand_ids, int* cand_cnt, void* stream) {
  return dmlp_screen_hl(KT, cap, 2, KT * 32, xfrag, xinit, n_tiles, qhi, qlo, qn, qidx, qk, nq,
                        xnmax_bits, bad, eps_rel, S, cand_ids, cand_cnt, stream);
}

extern "C" void dmlp_set_screen_mode(int mode) { g_screen_mode = mode; }

extern "C" int dmlp_screen_debug_counters(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_screen_dbg), sizeof(g_screen_dbg));
  if (e != hipSuccess) return -(int)e;
  if (reset) {
    unsigned long long z[8] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_screen_dbg), z, sizeof(z));
    if (e != hipSuccess) return -(int)e;
  }
  return 0;
}
