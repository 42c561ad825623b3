// screen.hip — the fused hot kernel: bf16x3 MFMA distance screen + streaming per-query
// threshold + candidate compaction (SURVEY.md §2.5 K2+K3, §7.4 H1/H2).
//
// Reference hot loop: for every (query, point) an exact fp64 distance and a heap/nth_element
// top-k (engine.cpp:235-256; bench_1 @0xcf38-0xd10c; bench_4 @0xcb80).  Exact fp64 costs
// 3 fp64 VALU ops per (pair, attribute); this kernel instead computes a SCORE
//     a(q,x) = <q-mu, x-mu> - |x-mu|^2 / 2   ( = (|q-mu|^2 - d(q,x)) / 2 )
// on the matrix cores with a 3-term bf16 split (hi*hi + hi*lo + lo*hi, fp32 accumulate;
// mfma_f32_16x16x32_bf16), then keeps, per query, every point whose score could still belong
// to the exact top-k.  With |a - a_exact| <= eps_q (rigorous bound, see knn.py) and a_k the
// k-th largest score buffered so far, every point with a < a_k - 2*eps_q is provably outside
// the exact top-k (and not even tied), so the per-query threshold h = a_k - 2*eps_q only rises.
// Survivors are re-ranked exactly (fp64, no FMA, reference order) by refine.hip, so the final
// neighbour lists and checksums are bit-identical to the reference.
//
// Geometry (gfx950): one workgroup = WAVES waves, each wave owns 16 queries (one MFMA column
// tile) for the whole stream; query bf16 fragments live in VGPRs.  The data slice streams
// through an NBUF-deep LDS ring in 64-point tiles staged with global_load_lds (1 KiB
// lane-linear fragments laid out by prep.hip), counted vmcnt + raw s_barrier so the DMA of
// tile i+NBUF-1 overlaps the MFMAs of tile i.  The per-query candidate buffers (CAP entries of
// {score, id}) sit in LDS; appends use LDS atomics and are rare after the first tiles.  When a
// buffer passes CAP-64 the owning wave compacts it alone (bitonic sort of the scores across the
// wave), so no workgroup-wide synchronisation is needed beyond the tile ring.
// Block -> (query block, data slice) is XCD-aware: with S % 8 == 0 every XCD streams only its
// own S/8 slices, so each slice is fetched into exactly one XCD's L2.
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>

namespace {

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int KT, int WAVES, int CAP, int NBUF>
struct ScreenCfg {
  static constexpr int FRAGS = 4 * KT * 2;          // 1 KiB fragments per tile
  static constexpr int TILE_BYTES = FRAGS * 1024 + 256;
  static constexpr int G = FRAGS / WAVES;           // glds per wave per tile (+1 for wave 0)
  static constexpr int LDS = NBUF * TILE_BYTES + WAVES * 16 * CAP * 8 + WAVES * 16 * 4;
  static_assert(FRAGS % WAVES == 0, "fragments must split evenly over waves");
  static_assert(LDS <= 163840, "LDS budget");
  static_assert(CAP % 64 == 0, "CAP multiple of 64");
};

template <int KT, int WAVES, int CAP, int NBUF>
__global__ __launch_bounds__(WAVES * 64, 1) void k_screen(
    const uint4* __restrict__ xfrag, const float* __restrict__ xinit, int n_tiles,
    const bf16x8* __restrict__ qhi, const bf16x8* __restrict__ qlo, const float* __restrict__ qn,
    const int* __restrict__ qidx, const int* __restrict__ qk, int nq,
    const unsigned* __restrict__ xnmax_bits, const unsigned* __restrict__ bad, float eps_rel,
    int S, int tiles_per_slice, int n_qblocks, int* __restrict__ cand_ids,
    int* __restrict__ cand_cnt) {
  using C = ScreenCfg<KT, WAVES, CAP, NBUF>;
  constexpr int E = CAP / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* tiles = smem;
  int2* bufs = (int2*)(smem + NBUF * C::TILE_BYTES);
  int* cnts = (int*)(smem + NBUF * C::TILE_BYTES + WAVES * 16 * CAP * 8);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c = lane & 15;       // MFMA column = query of this lane
  const int kg = lane >> 4;      // k-group / row group

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
  bf16x8 bh[KT], bl[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    bh[kt] = qhi[(q * KT + kt) * 4 + kg];
    bl[kt] = qlo[(q * KT + kt) * 4 + kg];
  }
  const float eps = eps_rel * (qn[q] + xnmax);
  const int kq = valid ? qk[q] : 0;
  float h = valid ? -FLT_MAX : INFINITY;

  int2* const wbuf = bufs + wave * 16 * CAP;
  int* const wcnt = cnts + wave * 16;
  if (lane < 16) wcnt[lane] = 0;
  wait_vmcnt<0>();

  // ---- tile staging (lane-linear 1 KiB fragments, global -> LDS DMA)
  auto issue = [&](int i) {
    int ti = i < nt ? i : (nt > 0 ? nt - 1 : 0);  // past the end: re-stage the last tile (keeps
    const int t = t0 + ti;                          // vmcnt bookkeeping constant)
    char* dst = tiles + (i % NBUF) * C::TILE_BYTES;
    const uint4* src = xfrag + (int64_t)t * (C::FRAGS * 64);
#pragma unroll
    for (int g = 0; g < C::G; ++g) {
      const int f = wave + g * WAVES;
      __builtin_amdgcn_global_load_lds((const void*)(src + f * 64 + lane), (lds_ptr_t)(dst + f * 1024),
                                       16, 0, 0);
    }
    if (wave == 0)
      __builtin_amdgcn_global_load_lds((const void*)(xinit + (int64_t)t * 64 + lane),
                                       (lds_ptr_t)(dst + C::FRAGS * 1024), 4, 0, 0);
  };

  // ---- wave-local compaction of column cc's buffer
  auto compact = [&](int cc) {
    int2* qbuf = wbuf + cc * CAP;
    const int n = wcnt[cc];
    int2 e[E];
    float v[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int idx = r * 64 + lane;
      e[r] = idx < n ? qbuf[idx] : make_int2(__float_as_int(-INFINITY), -1);
      v[r] = __int_as_float(e[r].x);
    }
    dmlp::wave_sort_desc<E>(v);
    const int kc = __shfl(kq, cc);
    const float ec = __shfl(eps, cc);
    const float ak = dmlp::wave_pick<E, float>(v, kc - 1);
    const float hn = ak - 2.0f * ec;
    if (c == cc) h = fmaxf(h, hn);
    const float hc = __shfl(h, cc);
    int base = 0;
    dmlp::wave_sync();
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int idx = r * 64 + lane;
      const bool keep = idx < n && __int_as_float(e[r].x) >= hc;
      const unsigned long long m = __ballot(keep);
      if (keep) qbuf[base + __popcll(m & dmlp::lanemask_lt())] = e[r];
      base += __popcll(m);
    }
    dmlp::wave_sync();
    if (base > CAP - 64) {  // pathological ties: give up on this query, exact fallback
      if (c == cc) h = INFINITY;
      base = -1;
    }
    if (lane == 0) wcnt[cc] = base;
    dmlp::wave_sync();
  };

  // ---- prologue
  if (nt > 0) {
#pragma unroll
    for (int i = 0; i < NBUF - 1; ++i) issue(i);
  }

  for (int i = 0; i < nt; ++i) {
    if (wave == 0) wait_vmcnt<(NBUF - 2) * (C::G + 1)>();
    else wait_vmcnt<(NBUF - 2) * C::G>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(i + NBUF - 1);

    const char* tb = tiles + (i % NBUF) * C::TILE_BYTES;
    f32x4 acc[4];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
      acc[rt] = *(const f32x4*)(tb + C::FRAGS * 1024 + rt * 64 + kg * 16);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
        const bf16x8 ahi = *(const bf16x8*)(tb + ((rt * KT + kt) * 2 + 0) * 1024 + lane * 16);
        const bf16x8 alo = *(const bf16x8*)(tb + ((rt * KT + kt) * 2 + 1) * 1024 + lane * 16);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bh[kt], acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bl[kt], acc[rt], 0, 0, 0);
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bh[kt], acc[rt], 0, 0, 0);
      }
    }
    float m = fmaxf(fmaxf(acc[0][0], acc[0][1]), fmaxf(acc[0][2], acc[0][3]));
#pragma unroll
    for (int rt = 1; rt < 4; ++rt)
      m = fmaxf(m, fmaxf(fmaxf(acc[rt][0], acc[rt][1]), fmaxf(acc[rt][2], acc[rt][3])));
    if (__ballot(m >= h)) {
      // rare path: append every passing (score, id) to its query's buffer
      const int idbase = (t0 + i) * 64 + kg * 4;
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (acc[rt][j] >= h) {
            const int pos = atomicAdd(&wcnt[c], 1);
            wbuf[c * CAP + pos] = make_int2(__float_as_int(acc[rt][j]), idbase + rt * 16 + j);
          }
        }
      }
      dmlp::wave_sync();
      const bool need = lane < 16 && wcnt[lane] > CAP - 64;
      unsigned long long nm = __ballot(need);
      while (nm) {
        const int cc = __ffsll((long long)nm) - 1;
        nm &= nm - 1;
        compact(cc);
      }
    }
  }
  wait_vmcnt<0>();

  // ---- write this slice's candidates
  for (int cc = 0; cc < 16; ++cc) {
    const int pp = pbase + cc;
    if (pp >= nq) break;
    const int n = wcnt[cc];
    int* out = cand_ids + ((int64_t)pp * S + s) * CAP;
    if (n < 0) {
      if (lane == 0) cand_cnt[(int64_t)pp * S + s] = -1;
      continue;
    }
    const float hc = __shfl(h, cc);
    const int2* qbuf = wbuf + cc * CAP;
    int base = 0;
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int idx = r * 64 + lane;
      int2 e = make_int2(0, -1);
      if (idx < n) e = qbuf[idx];
      const bool keep = idx < n && __int_as_float(e.x) >= hc;
      const unsigned long long m = __ballot(keep);
      if (keep) out[base + __popcll(m & dmlp::lanemask_lt())] = e.y;
      base += __popcll(m);
    }
    if (lane == 0) cand_cnt[(int64_t)pp * S + s] = base;
  }
}

template <int KT, int WAVES, int CAP, int NBUF>
int launch_screen(const void* xfrag, const float* xinit, int64_t n_tiles, const void* qhi,
                  const void* qlo, const float* qn, const int* qidx, const int* qk, int nq,
                  const unsigned* xnmax, const unsigned* bad, float eps_rel, int S,
                  int* cand_ids, int* cand_cnt, hipStream_t stream) {
  using C = ScreenCfg<KT, WAVES, CAP, NBUF>;
  auto kern = k_screen<KT, WAVES, CAP, NBUF>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       C::LDS);
    if (e != hipSuccess) return -(int)e;
    attr_set = true;
  }
  const int n_qblocks = (nq + WAVES * 16 - 1) / (WAVES * 16);
  const int tps = (int)((n_tiles + S - 1) / S);
  const int64_t grid = (int64_t)n_qblocks * S;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WAVES * 64), C::LDS, stream,
                     (const uint4*)xfrag, xinit, (int)n_tiles, (const bf16x8*)qhi,
                     (const bf16x8*)qlo, qn, qidx, qk, nq, xnmax, bad, eps_rel, S, tps,
                     n_qblocks, cand_ids, cand_cnt);
  DMLP_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// (KT, CAP) -> (WAVES, NBUF): LDS = NBUF*(8 KiB*KT + 256) + WAVES*16*CAP*8 <= 160 KiB.
#define DMLP_SCREEN_CONFIGS(X)                                                                  \
  X(1, 128, 8, 3) X(2, 128, 4, 3) X(3, 128, 4, 3) X(4, 128, 4, 2) X(1, 256, 4, 3)             \
  X(2, 256, 2, 3) X(3, 256, 2, 3) X(4, 256, 2, 2)

extern "C" int dmlp_screen_kmax(int cap) { return cap == 128 ? 32 : (cap == 256 ? 128 : 0); }

extern "C" int dmlp_screen_lds_bytes(int KT, int cap) {
#define DMLP_LDS_CASE(kt, cp, w, nb) \
  if (KT == kt && cap == cp) return ScreenCfg<kt, w, cp, nb>::LDS;
  DMLP_SCREEN_CONFIGS(DMLP_LDS_CASE)
#undef DMLP_LDS_CASE
  return -1;
}

extern "C" int dmlp_screen_waves(int KT, int cap) {
#define DMLP_W_CASE(kt, cp, w, nb) \
  if (KT == kt && cap == cp) return w;
  DMLP_SCREEN_CONFIGS(DMLP_W_CASE)
#undef DMLP_W_CASE
  return -1;
}

extern "C" int dmlp_screen(int KT, int cap, const void* xfrag, const float* xinit, int64_t n_tiles,
                           const void* qhi, const void* qlo, const float* qn, const int* qidx,
                           const int* qk, int nq, const unsigned* xnmax_bits, const unsigned* bad,
                           float eps_rel, int S, int* cand_ids, int* cand_cnt, void* stream) {
  if (nq <= 0) return 0;
  if (S < 1 || n_tiles < 0 || n_tiles > 0x7fffffff / 64) return -1;
  hipStream_t st = (hipStream_t)stream;
#define DMLP_SCREEN_CASE(kt, cp, w, nb)                                                        \
  if (KT == kt && cap == cp)                                                                   \
    return launch_screen<kt, w, cp, nb>(xfrag, xinit, n_tiles, qhi, qlo, qn, qidx, qk, nq,     \
                                        xnmax_bits, bad, eps_rel, S, cand_ids, cand_cnt, st);
  DMLP_SCREEN_CONFIGS(DMLP_SCREEN_CASE)
#undef DMLP_SCREEN_CASE
  return -2;
}
