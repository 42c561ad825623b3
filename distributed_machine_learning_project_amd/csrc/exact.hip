// exact.hip — fused streaming exact top-k (k <= 256): fp64 distances in the reference's order
// (engine.cpp:12-18: left to right over the attributes, each subtraction, product and sum
// separately rounded — no FMA) and the per-query selection in ONE pass, with no Q x N distance
// rows in HBM (fallback.hip writes every row, then radix-selects it: ~5 HBM passes per row).
//
// Workgroup = 256 threads = QB queries (64; 16 for k > 64); the data stream is tiled by 16 PJ
// points.  Thread (tx = tid & 15, ty = tid >> 4) owns the (QB/16) x PJ micro-tile of queries
// ty + 16 i and points tx + 16 j of the tile (query and point chunks staged in LDS), so a query's
// 16 threads all sit in ONE wave: every query's candidate buffer is wave-private and needs no
// workgroup barrier.  After a tile, its distances are offered in PJ rounds (one point column
// j per round, <= 16 candidates per query): a distance is appended iff it is <= the query's
// current threshold T (the k-th best so far; points arrive in increasing id order, so a later
// point equal to T — larger id — ranks before it under (dist asc, id desc) and must be kept).
// Before a round, if some buffer of the wave could overflow, the wave compacts: every entry's
// rank among its query's buffer (key_less, exact order), the best k rewritten in sorted order,
// T = the k-th.  At the end one compaction sorts every buffer and the first k go out.
#include "dmlp.h"
#include "dmlp_device.h"
#include <math.h>
#include <stdlib.h>

namespace {

// QB queries per workgroup (RI = QB / 16 rows per thread), PJ points per thread per tile
// (tile = 16 PJ points), CB candidate slots per query, AC attributes per LDS chunk.
template <int QB_, int PJ_, int CB_, int AC_, int WPE_ = 2>
struct Ex {
  static constexpr int QB = QB_, PJ = PJ_, PT = 16 * PJ_, CB = CB_, AC = AC_;
  static constexpr int WPE = WPE_;    // waves per SIMD the kernel is compiled for
  static constexpr int AS = AC + 2;   // LDS row stride in doubles: 16-byte aligned rows (b128)
  static constexpr int RI = QB / 16;  // rows (queries) per thread
  static constexpr int EPL = (CB + 63) / 64;  // buffer entries per lane in a compaction
  static constexpr int NQ = (QB * AC + 255) / 256, NX = (PT * AC + 255) / 256;
  static constexpr int STG = (QB + PT) * AS * 8;                    // Qs + Xs chunk staging
  static constexpr int BUF = QB * CB * (8 + 4) + QB * 4 + QB * 8;   // entries + counts + T
  static constexpr int LDS = STG + BUF;
};
using ExK16 = Ex<64, 8, 48, 16>;    // k <= 16: 2 workgroups per CU
// (measured and dropped: a 4x4 micro-tile with 32-slot buffers at 3 waves per SIMD — 73.5 ms
// against 54.1 ms, profiles/r4l_exact_variants.txt: the extra LDS reads per fp64 op cost more
// than the occupancy hides)
using ExK32 = Ex<64, 8, 64, 16>;
using ExK64 = Ex<64, 8, 128, 16>;
using ExK256 = Ex<16, 16, 384, 8>;  // k <= 256: 16 queries per workgroup, 384-slot buffers

// Compact every row of wave `wave` that holds more than its k entries (final: every row, and
// write the sorted first k out).  Rows of wave w: ty in [4w, 4w + 4) x i -> 4 RI rows.  Rare
// (a few times per query), so it is an out-of-line call: inlined at every offer round it
// would inflate the hot loop's register allocation.
template <class C>
__device__ __noinline__ void compact_rows(double* __restrict__ bd, int* __restrict__ bi,
                                          int* __restrict__ cnt, double* __restrict__ thr,
                                          const int* __restrict__ qidx,
                                          const int* __restrict__ qk, int nb, int64_t N, int q0,
                                          int wave, int lane, bool final_pass,
                                          double* __restrict__ out_d, int* __restrict__ out_i,
                                          int kstride) {
  constexpr int CB = C::CB, EPL = C::EPL;
  for (int s = 0; s < 4 * C::RI; ++s) {
    const int r = (4 * wave + (s & 3)) + 16 * (s >> 2);
    const int n = cnt[r];
    const int q = q0 + r;
    int k = 0;
    if (q < nb) {
      k = qk[qidx[q]];
      if ((int64_t)k > N) k = (int)N;
    }
    if (!final_pass && n <= k) continue;
    double* rd = bd + r * CB;
    int* ri = bi + r * CB;
    // ranks of this lane's entries (lane + 64 h) under (dist asc, id desc)
    double ed[EPL];
    int ei[EPL], rk[EPL];
#pragma unroll
    for (int h = 0; h < EPL; ++h) {
      const int e = lane + 64 * h;
      rk[h] = 1 << 30;
      if (e < n) {
        ed[h] = rd[e];
        ei[h] = ri[e];
        int c = 0;
        for (int j = 0; j < n; ++j) c += dmlp::key_less(rd[j], ri[j], ed[h], ei[h]) ? 1 : 0;
        rk[h] = c;
      }
    }
    dmlp::wave_sync();  // every lane has read the buffer before any rewrite
    const int kept = n < k ? n : k;
#pragma unroll
    for (int h = 0; h < EPL; ++h) {
      if (rk[h] < kept) {
        if (final_pass) {
          out_d[(int64_t)qidx[q] * kstride + rk[h]] = ed[h];
          out_i[(int64_t)qidx[q] * kstride + rk[h]] = ei[h];
        } else {
          rd[rk[h]] = ed[h];
          ri[rk[h]] = ei[h];
        }
      }
    }
    dmlp::wave_sync();
    if (lane == 0) {
      cnt[r] = kept;
      thr[r] = (!final_pass && kept == k && k > 0) ? rd[k - 1] : INFINITY;
    }
    dmlp::wave_sync();
  }
}

template <class C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(C::WPE))) void k_exact_topk(const double* __restrict__ X, int64_t N, int A,
                                                    const double* __restrict__ Qx,
                                                    const int* __restrict__ qidx,
                                                    const int* __restrict__ qk, int nb,
                                                    double* __restrict__ out_d,
                                                    int* __restrict__ out_i, int kstride) {
  constexpr int QB = C::QB, PJ = C::PJ, PT = C::PT, CB = C::CB, AC = C::AC, AS = C::AS;
  constexpr int RI = C::RI, NQ = C::NQ, NX = C::NX;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double (*Qs)[AS] = (double (*)[AS])smem;
  double (*Xs)[AS] = (double (*)[AS])(smem + QB * AS * 8);
  double* const bd = (double*)(smem + C::STG);                       // [QB][CB]
  int* const bi = (int*)(bd + QB * CB);                              // [QB][CB]
  int* const cnt = bi + QB * CB;                                     // [QB]
  double* const thr = (double*)(cnt + QB);                           // [QB]
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int lane = tid & 63, wave = tid >> 6;
  const int q0 = blockIdx.x * QB;
  // this thread's rows: ty + 16 i; per-row k (0 for rows past nb)
  int kq[RI];
  double tq[RI];
#pragma unroll
  for (int i = 0; i < RI; ++i) {
    const int r = ty + 16 * i;
    kq[i] = q0 + r < nb ? qk[qidx[q0 + r]] : 0;
    if ((int64_t)kq[i] > N) kq[i] = (int)N;
    tq[i] = INFINITY;
  }
  if (tid < QB) { cnt[tid] = 0; thr[tid] = INFINITY; }
  __syncthreads();

  // staging is software-pipelined: the next (tile, chunk)'s elements are loaded into registers
  // while the current chunk computes, so no wave waits on global memory at the barriers
  double qr[NQ], xr[NX];
  auto fetch = [&](int64_t p0, int a0) __attribute__((always_inline)) {
    const int ac = A - a0 < AC ? A - a0 : AC;
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int e = tid + 256 * u, r = e / AC, a = e % AC;
      const int qi = q0 + r;
      qr[u] = (e < QB * AC && qi < nb && a < ac) ? Qx[(int64_t)qidx[qi] * A + a0 + a] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int e = tid + 256 * u, r = e / AC, a = e % AC;
      const int64_t pi = p0 + r;
      xr[u] = (e < PT * AC && pi < N && a < ac) ? X[pi * A + a0 + a] : 0.0;
    }
  };
  fetch(0, 0);
  for (int64_t p0 = 0; p0 < N; p0 += PT) {
    double acc[RI][PJ];
#pragma unroll
    for (int i = 0; i < RI; ++i)
#pragma unroll
      for (int j = 0; j < PJ; ++j) acc[i][j] = 0.0;
    for (int a0 = 0; a0 < A; a0 += AC) {
      const int ac = A - a0 < AC ? A - a0 : AC;
      __syncthreads();  // the previous chunk's reads are done
#pragma unroll
      for (int u = 0; u < NQ; ++u)
        if (tid + 256 * u < QB * AC) Qs[(tid + 256 * u) / AC][(tid + 256 * u) % AC] = qr[u];
#pragma unroll
      for (int u = 0; u < NX; ++u)
        if (tid + 256 * u < PT * AC) Xs[(tid + 256 * u) / AC][(tid + 256 * u) % AC] = xr[u];
      __syncthreads();
      {
        int64_t np = p0;
        int na = a0 + AC;
        if (na >= A) { na = 0; np = p0 + PT; }
        if (np < N) fetch(np, na);
      }
      // two attributes per step: 16-byte LDS reads; the sums stay in attribute order
      int a = 0;
      for (; a + 1 < ac; a += 2) {
        double2 qv[RI], xv[PJ];
#pragma unroll
        for (int i = 0; i < RI; ++i) qv[i] = *(const double2*)&Qs[ty + 16 * i][a];
#pragma unroll
        for (int j = 0; j < PJ; ++j) xv[j] = *(const double2*)&Xs[tx + 16 * j][a];
#pragma unroll
        for (int i = 0; i < RI; ++i)
#pragma unroll
          for (int j = 0; j < PJ; ++j) {
            const double d0 = __dsub_rn(qv[i].x, xv[j].x);
            acc[i][j] = __dadd_rn(acc[i][j], __dmul_rn(d0, d0));
            const double d1 = __dsub_rn(qv[i].y, xv[j].y);
            acc[i][j] = __dadd_rn(acc[i][j], __dmul_rn(d1, d1));
          }
      }
      if (a < ac) {  // odd attribute count: the last one alone
        double qv[RI], xv[PJ];
#pragma unroll
        for (int i = 0; i < RI; ++i) qv[i] = Qs[ty + 16 * i][a];
#pragma unroll
        for (int j = 0; j < PJ; ++j) xv[j] = Xs[tx + 16 * j][a];
#pragma unroll
        for (int i = 0; i < RI; ++i)
#pragma unroll
          for (int j = 0; j < PJ; ++j) {
            const double d0 = __dsub_rn(qv[i], xv[j]);
            acc[i][j] = __dadd_rn(acc[i][j], __dmul_rn(d0, d0));
          }
      }
    }
    // offer the tile's distances, one point column per round (<= 16 per query per round)
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      bool full = false;
#pragma unroll
      for (int i = 0; i < RI; ++i) full |= cnt[ty + 16 * i] > CB - 16;
      if (__ballot(full)) {
        compact_rows<C>(bd, bi, cnt, thr, qidx, qk, nb, N, q0, wave, lane, false, out_d, out_i,
                         kstride);
#pragma unroll
        for (int i = 0; i < RI; ++i) tq[i] = thr[ty + 16 * i];
      }
      const int64_t p = p0 + tx + 16 * j;
#pragma unroll
      for (int i = 0; i < RI; ++i) {
        if (p < N && kq[i] > 0 && acc[i][j] <= tq[i]) {
          const int r = ty + 16 * i;
          const int pos = atomicAdd(&cnt[r], 1);
          bd[r * CB + pos] = acc[i][j];
          bi[r * CB + pos] = (int)p;
        }
      }
      dmlp::wave_sync();
    }
  }
  compact_rows<C>(bd, bi, cnt, thr, qidx, qk, nb, N, q0, wave, lane, true, out_d, out_i,
                   kstride);
}

template <class C>
int launch_exact(const double* X, int64_t N, int A, const double* Qx, const int* qidx,
                 const int* qk, int nb, double* out_d, int* out_i, int kstride, hipStream_t st) {
  const int lds = C::LDS;
  static const bool attr = hipFuncSetAttribute((const void*)&k_exact_topk<C>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               lds) == hipSuccess;
  if (!attr) return -5;
  hipLaunchKernelGGL((k_exact_topk<C>), dim3((unsigned)((nb + C::QB - 1) / C::QB)), dim3(256),
                     lds, st, X, N, A, Qx, qidx, qk, nb, out_d, out_i, kstride);
  DMLP_LAUNCH_CHECK();
  return 0;
}

}  // namespace

extern "C" int dmlp_exact_topk_kmax(void) { return 256; }
// The largest k the fused kernel should take for a dataset of N points.  For k in (64, 256] its
// rank-based compactions of 384-slot buffers cost about as much as the distances when N is
// small (N = 1e5, k = 200: 93.6 ms vs 23.5 ms for rows + radix select), and win once the
// rows' HBM traffic grows (N = 1e6: 260 vs 756 ms; N = 1e7: 1.5 s vs > 170 s).
extern "C" int dmlp_exact_topk_kmax_for(int64_t N) { return N >= (int64_t(1) << 19) ? 256 : 64; }

// Exact top-k (k <= 256, clamped to N) of queries qidx[0..nb), sorted by (dist asc, id desc) into
// out_*[q * kstride + j], j < k (slots past min(k, N) untouched).  kmax: an upper bound of the
// k of these queries (selects the buffer size).  No workspace.
extern "C" int dmlp_exact_topk(const double* X, int64_t N, int A, const double* Qx,
                               const int* qidx, const int* qk, int nb, int kmax, double* out_d,
                               int* out_i, int kstride, void* stream) {
  if (nb <= 0 || N <= 0) return 0;
  if (N > 0x7fffffff || A < 1 || kmax > 256) return -1;
  hipStream_t st = (hipStream_t)stream;
  if (kmax <= 16) return launch_exact<ExK16>(X, N, A, Qx, qidx, qk, nb, out_d, out_i, kstride, st);
  if (kmax <= 32) return launch_exact<ExK32>(X, N, A, Qx, qidx, qk, nb, out_d, out_i, kstride, st);
  if (kmax <= 64) return launch_exact<ExK64>(X, N, A, Qx, qidx, qk, nb, out_d, out_i, kstride, st);
  return launch_exact<ExK256>(X, N, A, Qx, qidx, qk, nb, out_d, out_i, kstride, st);
}
