// screen_f64.hip — the exact path's fp64 MFMA screen (v_mfma_f64_16x16x4_f64) + group refine.
//
// The fused exact kernel (exact.hip) spends 3 fp64 VALU operations per (query, point,
// attribute) — subtract, multiply, add, each rounded as the reference does (engine.cpp:12-18) —
// and runs at ~55 ms on the bench shape.  The same exact result needs the reference's rounding
// only for the few points that can still be in a query's top-k, so this path screens in fp64
// on the matrix cores and re-ranks the survivors with the reference's arithmetic:
//
//   score  s(q, x) = <q', x'> - |x'|^2 / 2   (x' = x - mu, q' = q - mu: centred for tightness)
//
// ranks points like -|q - x|^2 (d^2 = |q'|^2 - 2 s).  One wave owns 64 queries (4 column tiles)
// and streams 16-point steps of a slice of the dataset; per step and column tile it issues A/4
// fp64 MFMAs (K = 4), the C operand being -|x'|^2/2, so acc = s directly, accumulated in fp64.
// The candidate machinery is the single-term screen's (screen_x1.hip): 4-row group maxima become
// fp32 keys, appended to per-column LDS sub-buffers when they reach the column's threshold h,
// batched lane-parallel compactions raise h to (k-th largest group key) - 2 eps, and the final
// compaction writes the surviving group ids.  The group refine (refine.hip, E = 8, no rescoring)
// then takes every member of a group at or above the global threshold, computes the reference's
// exact distance for each and sorts: the output is bit-identical to exact.hip's.
//
// Error bound (eps per query, fp32): the fp64 score's error is at most gamma_{A+2} (|x'|^2/2 +
// |q'||x'|) in any summation order (u = 2^-53); the fp32 rounding of a group max adds 2^-24 |s|;
// the reference's own left-to-right rounding of d^2 moves a point's rank by at most
// gamma_{2A+1} d^2 / 2 in score units; centring in fp64 costs O(u (|q'| + |x'|)^2).  All of it is
// far below eps = 2^-20 (M^2/2 + |q'| M + (|q'| + M)^2), M = max |x'|, which also absorbs the
// fp32 arithmetic of the threshold update (hc = key - 2 eps).  Every true top-k member then
// keeps an fp32 group key >= hc at every compaction, as in screen_x1.hip's argument.
//
// Layout: the image permutes the 16 rows of a step so that lane (c, g) of the f64 MFMA — whose
// results are rows g, g+4, g+8, g+12 (cdna_hip_programming.md: f64 C/D col = lane & 15,
// row = (lane >> 4) + 4 reg) — holds points p0 + 4g .. p0 + 4g + 3: a contiguous 4-row group, so
// group ids mean what the refine expects (slice base + 4 * index + member).
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>

#include <cmath>

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned ord32f(unsigned b) {
  return b ^ ((unsigned)((int)b >> 31) | 0x80000000u);
}
__device__ __forceinline__ unsigned unord32f(unsigned o) {
  return o ^ ((o >> 31) ? 0x80000000u : 0xffffffffu);
}

// The step image: [step][c2 < NM/2][lane] double2 = x'[point(lane & 15)][4 (2 c2 + h) + (lane >> 4)]
// for h = 0, 1, where point(i) = p0 + 4 (i & 3) + (i >> 2) (zeros past N or A).
__global__ __launch_bounds__(256) void k_f64_image(const double* __restrict__ X, int64_t N, int A,
                                                   const double* __restrict__ mu, int NM,
                                                   int64_t n_steps, double2* __restrict__ frag) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int hm = NM >> 1;
  if (idx >= n_steps * hm * 64) return;
  const int lane = (int)(idx & 63);
  const int64_t rest = idx >> 6;
  const int c2 = (int)(rest % hm);
  const int64_t step = rest / hm;
  const int i = lane & 15, g = lane >> 4;
  const int64_t p = step * 16 + 4 * (i & 3) + (i >> 2);
  const int a0 = 4 * (2 * c2) + g, a1 = 4 * (2 * c2 + 1) + g;
  double v0 = 0.0, v1 = 0.0;
  if (p < N) {
    if (a0 < A) v0 = __dsub_rn(X[p * A + a0], mu[a0]);
    if (a1 < A) v1 = __dsub_rn(X[p * A + a1], mu[a1]);
  }
  frag[idx] = double2{v0, v1};
}

// -|x'|^2 / 2 per point (-inf past N: padding never reaches a threshold) and max |x'|^2 (fp64
// bits: non-negative doubles order like their bit patterns).
__global__ __launch_bounds__(256) void k_f64_norms(const double* __restrict__ X, int64_t N, int A,
                                                   const double* __restrict__ mu, int64_t n_pad,
                                                   double* __restrict__ xi,
                                                   unsigned long long* __restrict__ xnmax) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n_pad) return;
  double s = 0.0;
  if (p < N) {
    for (int a = 0; a < A; ++a) {
      const double d = __dsub_rn(X[p * A + a], mu[a]);
      s = __dadd_rn(s, __dmul_rn(d, d));
    }
    atomicMax(xnmax, (unsigned long long)__double_as_longlong(s));
  }
  xi[p] = p < N ? -0.5 * s : -INFINITY;
}

template <int NM, int SUB>
struct F64Cfg {
  static constexpr int CT = 4;
  static constexpr int NCOL = 64;
  static constexpr int CHECK = 2;
  static constexpr int CP = 4 * SUB + 4;
  static constexpr int CAPE = 4 * (SUB - CHECK);
  static constexpr int IDCAP = 4 * (SUB - 1);
  static constexpr int SBUF = NCOL * CP * 4;
  static constexpr int LDS = SBUF + NCOL * 4 * 4 + NCOL * 4 * 4;
};

template <int NM, int SUB>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SUB == 16 ? 2 : 1))) void k_screen_f64(
    const double2* __restrict__ frag, const double* __restrict__ xi, int n_tiles,
    const double* __restrict__ Qx, int A, const double* __restrict__ mu,
    const int* __restrict__ qidx, const int* __restrict__ qk, int nq,
    const unsigned long long* __restrict__ xnmax_bits, int S, int tiles_per_slice, int n_qblocks,
    int* __restrict__ cand_ids, int* __restrict__ cand_cnt, float* __restrict__ cand_h) {
  using C = F64Cfg<NM, SUB>;
  constexpr int CT = C::CT;
  constexpr int HM = NM / 2;  // 16-byte fragment loads per step
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned* const sbuf = (unsigned*)smem;
  int* const lcnt = (int*)(smem + C::SBUF);
  float* const lh = (float*)(lcnt + C::NCOL * 4);
  int* const lk = (int*)(lh + C::NCOL);
  float* const leps = (float*)(lk + C::NCOL);
  int* const lflag = (int*)(leps + C::NCOL);

  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const int kg = lane >> 4;

  const int b = blockIdx.x;
  int qb, s;
  if ((S & 7) == 0) {  // XCD-aware: slice s stays on one XCD's L2
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
  const int pbase = qb * C::NCOL;
  const double xn = __longlong_as_double((long long)*xnmax_bits);

  // query fragments (B operand): lane (c, kg) holds q'[col][4 m + kg]
  double bq[CT][NM];
  float h[CT];
  unsigned addr[CT], lim[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int p = pbase + ct * 16 + c;
    const bool valid = p < nq;
    const int q = valid ? qidx[p] : 0;
    double qq = 0.0;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      const int a = 4 * m + kg;
      bq[ct][m] = valid && a < A ? __dsub_rn(Qx[(int64_t)q * A + a], mu[a]) : 0.0;
      qq += bq[ct][m] * bq[ct][m];
    }
    qq += __shfl_xor(qq, 16);
    qq += __shfl_xor(qq, 32);
    // magnitudes past 1e30 (|s| near the fp32 key range, or inf / NaN): the column reports
    // overflow and the caller re-ranks it on the VALU kernel
    const bool big = !(qq < 1e30) || !(xn < 1e30);
    h[ct] = valid && !big ? -FLT_MAX : INFINITY;
    addr[ct] = (unsigned)(((ct * 16 + c) * C::CP + kg) * 4);
    lim[ct] = addr[ct] + (SUB - C::CHECK) * 16;
    if (lane < 16) {
      const int col = ct * 16 + c;
      lh[col] = h[ct];
      lk[col] = valid ? qk[q] : 0;
      const double qm = sqrt(qq), xm = sqrt(xn);
      const double e = 0x1p-20 * (0.5 * xn + qm * xm + (qm + xm) * (qm + xm)) + 1e-30;
      leps[col] = valid && !big ? (float)(e * 1.001) : 0.0f;
      lflag[col] = valid && big ? 1 : 0;
    }
  }
  const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(frag + (int64_t)t0 * 4 * HM * 64), (short)0, nt * 4 * HM * 64 * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(xi + (int64_t)t0 * 64), (short)0, nt * 64 * 8, 0x00020000);

  // ---- batched compaction (screen_x1.hip's, without the COLLECT / ablation modes): lane j owns
  // column j; FINAL writes the column's group ids
  auto compact = [&](const bool final_pass) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      lcnt[(ct * 16 + c) * 4 + kg] = (int)(addr[ct] - (lim[ct] - (SUB - C::CHECK) * 16)) >> 4;
    dmlp::wave_sync();
    {
      const int j = lane;
      unsigned* const colbuf = sbuf + j * C::CP;
      const int4 n4 = *(const int4*)(lcnt + j * 4);
      const int nm[4] = {n4.x, n4.y, n4.z, n4.w};
      const int kc = lk[j];
      const float epc = leps[j];
      const int flag = lflag[j];
      float hc = lh[j];
      unsigned e[4 * SUB];
      unsigned mx = 0u;
      const unsigned mn = ord32f(__float_as_uint(hc)) & 0xffff0000u;
#pragma unroll
      for (int v = 0; v < SUB; ++v) {
        const u32x4 raw = *(const u32x4*)(colbuf + 4 * v);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const unsigned vm = (unsigned)((v - nm[m]) >> 31);
          const unsigned o = ord32f(raw[m]) & vm;
          e[4 * v + m] = o;
          mx = max(mx, o);
        }
      }
      const int ntot = nm[0] + nm[1] + nm[2] + nm[3];
      const bool sel = !flag && kc >= 1 && ntot >= kc;
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
      T <<= 1;
      if (sel) {
        const float ak = __uint_as_float(unord32f(T << 16));
        hc = fmaxf(hc, ak - 2.0f * epc);
      }
      const unsigned kh = flag ? 0xffffffffu : ord32f(__float_as_uint(hc)) & 0xffff0000u;
      if (!final_pass) {
        int pos = 0;
#pragma unroll
        for (int i = 0; i < 4 * SUB; ++i) {
          const bool keep = e[i] >= kh;
          colbuf[keep ? pos : 4 * SUB] = unord32f(e[i]);
          pos += keep ? 1 : 0;
        }
        const bool ovf = flag || pos > C::CAPE;
        int4 nn;
        nn.x = ovf ? 0 : (pos + 3) >> 2;
        nn.y = ovf ? 0 : (pos + 2) >> 2;
        nn.z = ovf ? 0 : (pos + 1) >> 2;
        nn.w = ovf ? 0 : pos >> 2;
        *(int4*)(lcnt + j * 4) = nn;
        lh[j] = ovf ? INFINITY : hc;
        lflag[j] = ovf ? 1 : 0;
      } else {
        const int p = pbase + j;
        if (p < nq) {
          int* const out = cand_ids + ((int64_t)p * S + s) * C::IDCAP;
          int kept = 0;
#pragma unroll
          for (int i = 0; i < 4 * SUB; ++i) {
            const bool keep = e[i] >= kh;
            if (keep && kept < C::CAPE)
              out[kept] = (int)((e[i] & 0xffff0000u) | (unord32f(e[i]) & 0xffffu));
            kept += keep ? 1 : 0;
          }
          cand_cnt[(int64_t)p * S + s] = (flag || kept > C::CAPE) ? -1 : kept;
          cand_h[2 * ((int64_t)p * S + s)] = hc;
          cand_h[2 * ((int64_t)p * S + s) + 1] = epc;
        }
      }
    }
    if (!final_pass) {
      dmlp::wave_sync();
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        addr[ct] = lim[ct] - (SUB - C::CHECK) * 16 + 16 * lcnt[(ct * 16 + c) * 4 + kg];
        h[ct] = lh[ct * 16 + c];
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    }
  };

  // ---- 2-deep register ring of step fragments + double-buffered accumulators
  double2 fa[2][HM];
  f64x4 xr[2];
  f64x4 acc[2][CT];
  auto load = [&](int j, int r) __attribute__((always_inline)) {
#pragma unroll
    for (int h2 = 0; h2 < HM; ++h2)
      fa[r][h2] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                                                  fr, lane * 16, (j * HM + h2) * 1024, 0));
    const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(ir, kg * 32, j * 128, 0);
    const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(ir, kg * 32 + 16, j * 128, 0);
    const double2 l2 = __builtin_bit_cast(double2, lo), h2v = __builtin_bit_cast(double2, hi);
    xr[r] = f64x4{l2.x, l2.y, h2v.x, h2v.y};
  };
  auto mfma = [&](int r, int ab) __attribute__((always_inline)) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      f64x4 a = xr[r];
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const double av = (m & 1) ? fa[r][m >> 1].y : fa[r][m >> 1].x;
        a = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bq[ct][m], a, 0, 0, 0);
      }
      acc[ab][ct] = a;
    }
  };
  unsigned long long trig = 0;
  auto epilogue = [&](int ab, int J) __attribute__((always_inline)) {
    float m32[CT];
    bool hit[CT];
    bool any = false;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const double mm = fmax(fmax(acc[ab][ct][0], acc[ab][ct][1]), fmax(acc[ab][ct][2], acc[ab][ct][3]));
      m32[ct] = (float)mm;
      hit[ct] = m32[ct] >= h[ct];
      any |= hit[ct];
    }
    if (__ballot(any)) {
      const unsigned gl = (unsigned)(J * 4 + kg);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        *(__attribute__((address_space(3))) unsigned*)(size_t)addr[ct] =
            (__float_as_uint(m32[ct]) & 0xffff0000u) | gl;
        addr[ct] += hit[ct] ? 16u : 0u;
        trig |= __ballot(addr[ct] > lim[ct]);
      }
    }
  };

  if (nsteps > 0) {
    load(0, 0);
    for (int j0 = 0; j0 < nsteps; j0 += 2) {  // nsteps is a multiple of 4
      load(j0 + 1, 1);
      mfma(0, 0);
      if (j0 > 0) epilogue(1, j0 - 1);
      load(j0 + 2, 0);  // past the slice: the buffer resource returns zeros
      mfma(1, 1);
      epilogue(0, j0);
      if (trig) compact(false);
      trig = 0;
    }
    epilogue(1, nsteps - 1);
  }
  compact(true);
}

// sub-buffer depth: 16 (two waves per SIMD) for k <= 16 up to A = 32; A in (32, 64] keeps its
// 12 / 16 query fragments per column tile in registers only at one wave per SIMD (512 registers:
// the two-wave form spills 184 / 340 bytes per lane), so it always takes the 32-deep form
int f64_sub(int kmax, int NM) { return kmax <= 16 && NM <= 8 ? 16 : 32; }

template <int NM, int SUB>
int launch_f64(const double2* frag, const double* xi, int64_t n_tiles, const double* Qx, int A,
               const double* mu, const int* qidx, const int* qk, int nq,
               const unsigned long long* xnmax, int S, int* cand_ids, int* cand_cnt,
               float* cand_h, hipStream_t st) {
  using C = F64Cfg<NM, SUB>;
  const int n_qblocks = (nq + C::NCOL - 1) / C::NCOL;
  const int tps = (int)((n_tiles + S - 1) / S);
  const int64_t grid = (int64_t)n_qblocks * S;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL((k_screen_f64<NM, SUB>), dim3((unsigned)grid), dim3(64), C::LDS, st, frag, xi,
                     (int)n_tiles, Qx, A, mu, qidx, qk, nq, xnmax, S, tps, n_qblocks, cand_ids,
                     cand_cnt, cand_h);
  DMLP_LAUNCH_CHECK();
  return 0;
}

int f64_nm(int A) { return A <= 8 ? 2 : A <= 16 ? 4 : A <= 32 ? 8 : A <= 48 ? 12 : A <= 64 ? 16 : 0; }

// Slices so that the grid fills 2 waves per SIMD (1024 SIMDs) with at most 4096 tiles (2^16
// groups) per slice and at most 256 slices (the refine's prefix array).
int f64_slices(int nq, int64_t n_tiles) {
  const int nqb = (nq + 63) / 64;
  int S = (int)std::max<int64_t>(1, std::min<int64_t>(n_tiles, (2048 + nqb - 1) / nqb));
  S = std::max<int>(S, (int)((n_tiles + 4095) / 4096));
  if (S > 8) S = (S + 7) & ~7;  // XCD-aware block mapping
  return std::min(S, 256);
}

struct F64Ws {
  double* mu;
  unsigned long long* xnmax;
  double2* frag;
  double* xi;
  int* cand_ids;
  int* cand_cnt;
  float* cand_h;
  int* ovf;
  int64_t bytes;
};

F64Ws f64_ws(char* base, int64_t N, int A, int nq, int kmax) {
  const int NM = f64_nm(A);
  const int64_t n_tiles = (N + 63) / 64;
  const int S = f64_slices(nq, n_tiles);
  const int idcap = 4 * (f64_sub(kmax, NM) - 1);
  auto al = [](int64_t x) { return (x + 255) & ~int64_t(255); };
  F64Ws w{};
  int64_t o = 0;
  w.mu = (double*)(base + o); o += al(8 * (int64_t)A);
  w.xnmax = (unsigned long long*)(base + o); o += al(8);
  w.ovf = (int*)(base + o); o += al(4);
  w.frag = (double2*)(base + o); o += al(n_tiles * 64 * (int64_t)NM * 4 * 8);  // 4 NM fp64 per point
  w.xi = (double*)(base + o); o += al(n_tiles * 64 * 8);
  w.cand_ids = (int*)(base + o); o += al((int64_t)nq * S * idcap * 4);
  w.cand_cnt = (int*)(base + o); o += al((int64_t)nq * S * 4);
  w.cand_h = (float*)(base + o); o += al((int64_t)nq * S * 8);
  w.bytes = o;
  return w;
}

// Layout probe (tests): scores of queries Qx[0..16) against points [0, 16) computed exactly as
// k_screen_f64 does (image, C operand, f64 MFMA chain, result rows g + 4r -> point 4g + r),
// written out[query * 16 + point].  NM = A padded / 4 (<= 16).
__global__ void k_f64_probe(const double2* __restrict__ frag, const double* __restrict__ xi,
                            const double* __restrict__ Qx, int A, const double* __restrict__ mu,
                            int NM, double* __restrict__ out) {
  const int lane = threadIdx.x & 63, c = lane & 15, kg = lane >> 4;
  f64x4 a;
  for (int r = 0; r < 4; ++r) a[r] = xi[4 * kg + r];
  for (int m = 0; m < NM; ++m) {
    const double2 v = frag[(m >> 1) * 64 + lane];
    const double av = (m & 1) ? v.y : v.x;
    const int at = 4 * m + kg;
    const double bv = at < A ? __dsub_rn(Qx[c * A + at], mu[at]) : 0.0;
    a = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, a, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) out[c * 16 + 4 * kg + r] = a[r];
}

}  // namespace

extern "C" int dmlp_exact_f64_probe(const double* X, int64_t N, int A, const double* Qx,
                                    double* out16x16, void* ws, int64_t ws_bytes, void* stream) {
  const int NM = f64_nm(A);
  if (NM == 0 || N < 16) return -3;
  F64Ws w = f64_ws((char*)ws, N, A, 64, 16);
  if (!ws || ws_bytes < w.bytes) return -1;
  hipStream_t st = (hipStream_t)stream;
  const int64_t n_tiles = (N + 63) / 64;
  int rc = dmlp_center(X, N, A, w.mu, stream);
  if (rc) return rc;
  if (hipMemsetAsync(w.xnmax, 0, 8, st) != hipSuccess) return -1;
  const int64_t n_steps = n_tiles * 4;
  const int64_t nimg = n_steps * (NM / 2) * 64;
  hipLaunchKernelGGL(k_f64_image, dim3((unsigned)((nimg + 255) / 256)), dim3(256), 0, st, X, N, A,
                     w.mu, NM, n_steps, w.frag);
  hipLaunchKernelGGL(k_f64_norms, dim3((unsigned)((n_tiles * 64 + 255) / 256)), dim3(256), 0, st,
                     X, N, A, w.mu, n_tiles * 64, w.xi, w.xnmax);
  hipLaunchKernelGGL(k_f64_probe, dim3(1), dim3(64), 0, st, w.frag, w.xi, Qx, A, w.mu, NM, out16x16);
  DMLP_LAUNCH_CHECK();
  return 0;
}
// Workspace layout (debugging): [0] S, [1] tiles per slice, [2] ids per (query, slice), byte
// offsets of [3] cand_ids, [4] cand_cnt, [5] cand_h, [6] xnmax, [7] mu.
extern "C" void dmlp_exact_f64_layout(int64_t N, int A, int nq, int kmax, int64_t* out) {
  F64Ws w = f64_ws(nullptr, N, A, nq, kmax);
  const int64_t n_tiles = (N + 63) / 64;
  const int S = f64_slices(nq, n_tiles);
  out[0] = S;
  out[1] = (n_tiles + S - 1) / S;
  out[2] = 4 * (f64_sub(kmax, f64_nm(A)) - 1);
  out[3] = (int64_t)(size_t)w.cand_ids;
  out[4] = (int64_t)(size_t)w.cand_cnt;
  out[5] = (int64_t)(size_t)w.cand_h;
  out[6] = (int64_t)(size_t)w.xnmax;
  out[7] = (int64_t)(size_t)w.mu;
}


extern "C" int dmlp_refine_groups_exact(int cap, const int* cand_ids, const int* cand_cnt,
                                        const float* cand_h, int S, int64_t tiles_per_slice,
                                        const double* X, int A, const double* Qx, int64_t n_points,
                                        const int* qidx, const int* qk, int nq, double* out_d,
                                        int* out_i, int kstride, int* status, int* ovf_count,
                                        void* stream);

// Largest A / k the fp64 screen serves (A: the query fragments live in registers).
extern "C" int dmlp_exact_f64_amax(void) { return 64; }
extern "C" int dmlp_exact_f64_kmax(void) { return 64; }

extern "C" int64_t dmlp_exact_f64_bytes(int64_t N, int A, int nq, int kmax) {
  if (f64_nm(A) == 0 || kmax > 64 || N <= 0 || nq <= 0) return 0;
  return f64_ws(nullptr, N, A, nq, kmax).bytes;
}

// Exact top-k of queries qidx[0..nq) (k <= 64, A <= 64): out_*[q * kstride + j], j < k, sorted by
// (dist asc, id desc), bit-identical to dmlp_exact_topk.  A query whose candidates overflow gets
// status[q] = 1 and nothing written (the caller runs dmlp_exact_topk on it); *ovf_count (device)
// is ADDED the number of them.  ws: dmlp_exact_f64_bytes(N, A, nq, kmax) bytes.
extern "C" int dmlp_exact_f64(const double* X, int64_t N, int A, const double* Qx, const int* qidx,
                              const int* qk, int nq, int kmax, double* out_d, int* out_i,
                              int kstride, int* status, int* ovf_count, void* ws, int64_t ws_bytes,
                              void* stream) {
  if (nq <= 0) return 0;
  const int NM = f64_nm(A);
  if (NM == 0 || kmax > 64 || kmax < 1 || N <= 0 || N > 0x7fffffff / 2) return -3;
  F64Ws w = f64_ws((char*)ws, N, A, nq, kmax);
  if (!ws || ws_bytes < w.bytes) return -1;
  hipStream_t st = (hipStream_t)stream;
  const int64_t n_tiles = (N + 63) / 64;
  const int S = f64_slices(nq, n_tiles);
  int rc = dmlp_center(X, N, A, w.mu, stream);
  if (rc) return rc;
  if (hipMemsetAsync(w.xnmax, 0, 8, st) != hipSuccess) return -1;
  const int64_t n_steps = n_tiles * 4;
  const int64_t nimg = n_steps * (NM / 2) * 64;
  hipLaunchKernelGGL(k_f64_image, dim3((unsigned)((nimg + 255) / 256)), dim3(256), 0, st, X, N, A,
                     w.mu, NM, n_steps, w.frag);
  DMLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_f64_norms, dim3((unsigned)((n_tiles * 64 + 255) / 256)), dim3(256), 0, st,
                     X, N, A, w.mu, n_tiles * 64, w.xi, w.xnmax);
  DMLP_LAUNCH_CHECK();
  const int sub = f64_sub(kmax, NM);
#define DMLP_F64(NMV)                                                                          \
  rc = sub == 16 ? launch_f64<NMV, 16>(w.frag, w.xi, n_tiles, Qx, A, w.mu, qidx, qk, nq, w.xnmax, S, \
                                       w.cand_ids, w.cand_cnt, w.cand_h, st)                  \
                 : launch_f64<NMV, 32>(w.frag, w.xi, n_tiles, Qx, A, w.mu, qidx, qk, nq, w.xnmax, S, \
                                       w.cand_ids, w.cand_cnt, w.cand_h, st)
  if (NM == 2) DMLP_F64(2);
  else if (NM == 4) DMLP_F64(4);
  else if (NM == 8) DMLP_F64(8);
  else if (NM == 12)
    rc = launch_f64<12, 32>(w.frag, w.xi, n_tiles, Qx, A, w.mu, qidx, qk, nq, w.xnmax, S,
                            w.cand_ids, w.cand_cnt, w.cand_h, st);
  else
    rc = launch_f64<16, 32>(w.frag, w.xi, n_tiles, Qx, A, w.mu, qidx, qk, nq, w.xnmax, S,
                            w.cand_ids, w.cand_cnt, w.cand_h, st);
#undef DMLP_F64
  if (rc) return rc;
  if (getenv("DMLP_EXACT_F64_SCREEN_ONLY")) return 0;  // debugging: the candidates stay in ws
  return dmlp_refine_groups_exact(4 * (sub - 1), w.cand_ids, w.cand_cnt, w.cand_h, S,
                                  (n_tiles + S - 1) / S, X, A, Qx, N, qidx, qk, nq, out_d, out_i,
                                  kstride, status, ovf_count, stream);
}
