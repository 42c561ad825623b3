// prep.hip — K1: layout transforms feeding the bf16x3 MFMA screen.
//
// The reference packs AoS vector<DataPoint> into flat arrays on rank 0 (engine.cpp:79-96,
// bench_1 @0xe1b0).  Here the flat fp64 rows are already on the GPU; this pass converts them
// ONCE per KNN call into the exact register image the MFMA A-operand wants, so the screen
// kernel's staging is a straight lane-linear global_load_lds of 1 KiB fragments:
//
//   tile t (64 points) = [rt 0..3][kt 0..KT-1][hl 0..1][lane 0..63][8 x bf16]
//   lane l of fragment (rt,kt,hl) holds point t*64 + rt*16 + (l&15),
//   attributes kt*32 + (l>>4)*8 + j, j = 0..7  (mfma_f32_16x16x32_bf16 A map).
//   hl = 0: hi = bf16(x - mu), hl = 1: lo = bf16((x - mu) - hi).
//   xinit[t*64 + r] = -(|x-mu|^2)/2 in fp32 (the MFMA C-init; -inf for padding rows).
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <chrono>
#include <vector>

namespace {

constexpr double kMaxAbs = 1.0e15;  // |x - mu| bound for the screen's fp32 range analysis

__device__ __forceinline__ unsigned short bf16_rn_bits(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32, round-to-nearest-even
  return __builtin_bit_cast(unsigned short, b);
}

// hi/lo split: hi = bf16(c), lo = bf16(c - hi) with c - hi exact in fp64.
__device__ __forceinline__ void split_bf16(double c, unsigned short& hi, unsigned short& lo) {
  const float cf = (float)c;
  hi = bf16_rn_bits(cf);
  const float hf = __uint_as_float(((unsigned)hi) << 16);
  const double r = c - (double)hf;
  lo = bf16_rn_bits((float)r);
}

// One block per attribute; deterministic tree reduction over the first min(N, 4096) rows.
__global__ void k_center(const double* __restrict__ X, int64_t N, int A, double* __restrict__ mu) {
  __shared__ double red[256];
  const int a = blockIdx.x;
  const int64_t n = N < 4096 ? N : 4096;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += X[i * A + a];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) mu[a] = n > 0 ? red[0] / (double)n : 0.0;
}

// One thread per (point, 8-attribute group).
__global__ void k_prep_frag(const double* __restrict__ X, int64_t N, int A,
                            const double* __restrict__ mu, int KT, int64_t n_tiles,
                            uint4* __restrict__ frag, unsigned* __restrict__ bad) {
  const int groups = KT * 4;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = n_tiles * 64 * groups;
  if (gid >= total) return;
  const int64_t p = gid / groups;
  const int g = (int)(gid - p * groups);
  const int kt = g >> 2, kg = g & 3;
  const int64_t t = p >> 6;
  const int pl = (int)(p & 63);
  const int rt = pl >> 4, r = pl & 15;
  const int lane = r + 16 * kg;
  unsigned short hi[8], lo[8];
  unsigned badv = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int a = kt * 32 + kg * 8 + j;
    double c = 0.0;
    if (p < N && a < A) {
      const double x = X[p * A + a];
      c = x - mu[a];
      if (!(fabs(c) < kMaxAbs)) { badv = 1; c = 0.0; }
    }
    split_bf16(c, hi[j], lo[j]);
  }
  if (badv) atomicOr(bad, 1u);
  const int64_t fbase = t * (int64_t)(4 * KT * 2) * 64;  // in uint4 (16 B) units
  const int64_t f_hi = fbase + (int64_t)((rt * KT + kt) * 2 + 0) * 64 + lane;
  const int64_t f_lo = fbase + (int64_t)((rt * KT + kt) * 2 + 1) * 64 + lane;
  uint4 vh, vl;
  vh.x = hi[0] | ((unsigned)hi[1] << 16); vh.y = hi[2] | ((unsigned)hi[3] << 16);
  vh.z = hi[4] | ((unsigned)hi[5] << 16); vh.w = hi[6] | ((unsigned)hi[7] << 16);
  vl.x = lo[0] | ((unsigned)lo[1] << 16); vl.y = lo[2] | ((unsigned)lo[3] << 16);
  vl.z = lo[4] | ((unsigned)lo[5] << 16); vl.w = lo[6] | ((unsigned)lo[7] << 16);
  frag[f_hi] = vh;
  frag[f_lo] = vl;
}

// Fragments + norms in one pass: one thread per (point, 8-attribute group) as in k_prep_frag;
// the G = 4*KT threads of a point are adjacent lanes, so |x - mu|^2 is a G-lane xor-shuffle
// reduction and every thread keeps its 8 centred values in registers (the row is read once).
// G must be a power of two (KT = 1, 2, 4, 8); the wave folds its max norm before the one atomic.
template <int G>
__global__ __launch_bounds__(256) void k_prep_frag_norm(const double* __restrict__ X, int64_t N,
                                                       int A, const double* __restrict__ mu,
                                                       int64_t n_tiles, uint4* __restrict__ frag,
                                                       float* __restrict__ xinit,
                                                       unsigned* __restrict__ xnmax_bits,
                                                       unsigned* __restrict__ bad) {
  constexpr int KT = G / 4;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = n_tiles * 64 * G;
  const bool live = gid < total;
  const int64_t p = gid / G;
  const int g = (int)(gid - p * G);
  const int kt = g >> 2, kg = g & 3;
  const int64_t t = p >> 6;
  const int pl = (int)(p & 63);
  const int rt = pl >> 4, r = pl & 15;
  const int lane = r + 16 * kg;
  unsigned short hi[8], lo[8];
  unsigned badv = 0;
  double ss = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int a = kt * 32 + kg * 8 + j;
    double c = 0.0;
    if (live && p < N && a < A) {
      c = X[p * A + a] - mu[a];
      if (!(fabs(c) < kMaxAbs)) { badv = 1; c = 0.0; }
    }
    ss += c * c;
    split_bf16(c, hi[j], lo[j]);
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1) ss += __shfl_xor(ss, o);
  if (badv) atomicOr(bad, 1u);
  if (live) {
    const int64_t fbase = t * (int64_t)(4 * KT * 2) * 64;  // in uint4 (16 B) units
    uint4 vh, vl;
    vh.x = hi[0] | ((unsigned)hi[1] << 16); vh.y = hi[2] | ((unsigned)hi[3] << 16);
    vh.z = hi[4] | ((unsigned)hi[5] << 16); vh.w = hi[6] | ((unsigned)hi[7] << 16);
    vl.x = lo[0] | ((unsigned)lo[1] << 16); vl.y = lo[2] | ((unsigned)lo[3] << 16);
    vl.z = lo[4] | ((unsigned)lo[5] << 16); vl.w = lo[6] | ((unsigned)lo[7] << 16);
    frag[fbase + (int64_t)((rt * KT + kt) * 2 + 0) * 64 + lane] = vh;
    frag[fbase + (int64_t)((rt * KT + kt) * 2 + 1) * 64 + lane] = vl;
  }
  // round the max up so the bound stays conservative; padding rows score -inf
  const float sf = (float)ss;
  float up = (live && p < N) ? sf * (1.0f + 1.0e-6f) + 1.0e-30f : 0.0f;
  if (live && g == 0) xinit[p] = p < N ? (float)(-0.5 * ss) : -INFINITY;
  // block max (non-negative floats order as their bits), one atomic per 256 threads
  __shared__ unsigned smax;
  if (threadIdx.x == 0) smax = 0u;
  __syncthreads();
  if (g == 0 && up > 0.0f) atomicMax(&smax, __float_as_uint(up));
  __syncthreads();
  if (threadIdx.x == 0 && smax) atomicMax(xnmax_bits, smax);
}

// One thread per point: xinit and the running max norm.
__global__ void k_prep_norm(const double* __restrict__ X, int64_t N, int A,
                            const double* __restrict__ mu, int64_t n_pad,
                            float* __restrict__ xinit, unsigned* __restrict__ xnmax_bits) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pad) return;
  if (p >= N) { xinit[p] = -INFINITY; return; }
  double s = 0.0;
  for (int a = 0; a < A; ++a) {
    double c = X[p * A + a] - mu[a];
    if (!(fabs(c) < kMaxAbs)) c = 0.0;
    s += c * c;
  }
  xinit[p] = (float)(-0.5 * s);
  // round the max up so the bound stays conservative
  const float sf = (float)s;
  const float up = sf * (1.0f + 1.0e-6f) + 1.0e-30f;
  atomicMax(xnmax_bits, __float_as_uint(up));
}

// One thread per (query, 8-attribute group), G = 4*KT adjacent lanes per query (power of two).
template <int G>
__global__ __launch_bounds__(256) void k_prep_queries_g(const double* __restrict__ Qx, int64_t Q,
                                                       int A, const double* __restrict__ mu,
                                                       uint4* __restrict__ qhi,
                                                       uint4* __restrict__ qlo,
                                                       float* __restrict__ qn,
                                                       unsigned* __restrict__ bad) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t q = gid / G;
  const int g = (int)(gid - q * G);
  const bool live = q < Q;
  unsigned short hi[8], lo[8];
  unsigned badv = 0;
  double ss = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int a = g * 8 + j;
    double c = 0.0;
    if (live && a < A) {
      c = Qx[q * A + a] - mu[a];
      if (!(fabs(c) < kMaxAbs)) { badv = 1; c = 0.0; }
    }
    ss += c * c;
    split_bf16(c, hi[j], lo[j]);
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1) ss += __shfl_xor(ss, o);
  if (badv) atomicOr(bad, 1u);
  if (!live) return;
  uint4 vh, vl;
  vh.x = hi[0] | ((unsigned)hi[1] << 16); vh.y = hi[2] | ((unsigned)hi[3] << 16);
  vh.z = hi[4] | ((unsigned)hi[5] << 16); vh.w = hi[6] | ((unsigned)hi[7] << 16);
  vl.x = lo[0] | ((unsigned)lo[1] << 16); vl.y = lo[2] | ((unsigned)lo[3] << 16);
  vl.z = lo[4] | ((unsigned)lo[5] << 16); vl.w = lo[6] | ((unsigned)lo[7] << 16);
  qhi[q * G + g] = vh;
  qlo[q * G + g] = vl;
  if (g == 0) qn[q] = (float)ss;
}

__global__ void k_prep_queries(const double* __restrict__ Qx, int64_t Q, int A,
                               const double* __restrict__ mu, int KT,
                               unsigned short* __restrict__ qhi, unsigned short* __restrict__ qlo,
                               float* __restrict__ qn, unsigned* __restrict__ bad) {
  const int64_t q = (int64_t)blockIdx.x;
  if (q >= Q) return;
  const int W = KT * 32;
  __shared__ double red[256];
  double s = 0.0;
  unsigned badv = 0;
  for (int a = threadIdx.x; a < W; a += blockDim.x) {
    double c = 0.0;
    if (a < A) {
      c = Qx[q * A + a] - mu[a];
      if (!(fabs(c) < kMaxAbs)) { badv = 1; c = 0.0; }
    }
    unsigned short h, l;
    split_bf16(c, h, l);
    qhi[q * W + a] = h;
    qlo[q * W + a] = l;
    s += c * c;
  }
  if (badv) atomicOr(bad, 1u);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = blockDim.x / 2; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) qn[q] = (float)red[0];
}

}  // namespace

extern "C" int dmlp_center(const double* X, int64_t N, int A, double* mu, void* stream) {
  if (A <= 0) return 0;
  hipLaunchKernelGGL(k_center, dim3(A), dim3(256), 0, (hipStream_t)stream, X, N, A, mu);
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int dmlp_prep_data(const double* X, int64_t N, int A, const double* mu, int KT,
                              void* xfrag, float* xinit, unsigned* xnmax_bits, unsigned* bad,
                              void* stream) {
  if (KT < 1 || A > KT * 32) return -1;
  const int64_t n_tiles = (N + 63) / 64;
  const int64_t total = n_tiles * 64 * KT * 4;
  if (total > 0 && (KT == 1 || KT == 2 || KT == 4 || KT == 8)) {
    const dim3 grid((unsigned)((total + 255) / 256));
    hipStream_t st = (hipStream_t)stream;
    if (KT == 1)
      hipLaunchKernelGGL(k_prep_frag_norm<4>, grid, dim3(256), 0, st, X, N, A, mu, n_tiles,
                         (uint4*)xfrag, xinit, xnmax_bits, bad);
    else if (KT == 2)
      hipLaunchKernelGGL(k_prep_frag_norm<8>, grid, dim3(256), 0, st, X, N, A, mu, n_tiles,
                         (uint4*)xfrag, xinit, xnmax_bits, bad);
    else if (KT == 4)
      hipLaunchKernelGGL(k_prep_frag_norm<16>, grid, dim3(256), 0, st, X, N, A, mu, n_tiles,
                         (uint4*)xfrag, xinit, xnmax_bits, bad);
    else
      hipLaunchKernelGGL(k_prep_frag_norm<32>, grid, dim3(256), 0, st, X, N, A, mu, n_tiles,
                         (uint4*)xfrag, xinit, xnmax_bits, bad);
    DMLP_LAUNCH_CHECK();
  } else if (total > 0) {
    const int64_t blocks = (total + 255) / 256;
    hipLaunchKernelGGL(k_prep_frag, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, X,
                       N, A, mu, KT, n_tiles, (uint4*)xfrag, bad);
    DMLP_LAUNCH_CHECK();
    const int64_t n_pad = n_tiles * 64;
    hipLaunchKernelGGL(k_prep_norm, dim3((unsigned)((n_pad + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, X, N, A, mu, n_pad, xinit, xnmax_bits);
    DMLP_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int dmlp_prep_queries(const double* Qx, int64_t Q, int A, const double* mu, int KT,
                                 void* qhi, void* qlo, float* qn, unsigned* bad, void* stream) {
  if (KT < 1 || A > KT * 32) return -1;
  if (Q <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (KT == 1 || KT == 2 || KT == 4 || KT == 8) {
    const int64_t total = Q * KT * 4;
    const dim3 grid((unsigned)((total + 255) / 256));
    if (KT == 1)
      hipLaunchKernelGGL(k_prep_queries_g<4>, grid, dim3(256), 0, st, Qx, Q, A, mu, (uint4*)qhi,
                         (uint4*)qlo, qn, bad);
    else if (KT == 2)
      hipLaunchKernelGGL(k_prep_queries_g<8>, grid, dim3(256), 0, st, Qx, Q, A, mu, (uint4*)qhi,
                         (uint4*)qlo, qn, bad);
    else if (KT == 4)
      hipLaunchKernelGGL(k_prep_queries_g<16>, grid, dim3(256), 0, st, Qx, Q, A, mu, (uint4*)qhi,
                         (uint4*)qlo, qn, bad);
    else
      hipLaunchKernelGGL(k_prep_queries_g<32>, grid, dim3(256), 0, st, Qx, Q, A, mu, (uint4*)qhi,
                         (uint4*)qlo, qn, bad);
    DMLP_LAUNCH_CHECK();
    return 0;
  }
  hipLaunchKernelGGL(k_prep_queries, dim3((unsigned)Q), dim3(64), 0, st, Qx, Q,
                     A, mu, KT, (unsigned short*)qhi, (unsigned short*)qlo, qn, bad);
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int dmlp_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Page-lock an existing host range (e.g. a node-shared /dev/shm mapping) so H2D copies from it
// run as DMA at full PCIe rate.  Returns 0 or the hipError_t code.
extern "C" int dmlp_host_register(void* p, int64_t bytes) {
  if (!p || bytes <= 0) return 0;
  return (int)hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault);
}

extern "C" int dmlp_host_unregister(void* p) {
  if (!p) return 0;
  return (int)hipHostUnregister(p);
}

// Host render + H2D of the screen operands, the dataset part restricted to tiles [t0, t1): host
// staging is indexed by absolute tile (the whole image's layout), the device image destinations
// xhi_d / xin_d point at the slot of tile t0 (a per-rank shard buffer that a collective then
// completes).  *xnm_d gets this range's max norm; if the range holds data outside the screen's
// range (return bit 1) it gets +inf instead, so a max-reduce over ranks tells every rank.
// (rows: X / Qx row-major, or — Xr / Qr non-null — tables of row pointers)
static int host_ops_h2d_tiles(const double* X, const double* const* Xr, int64_t N, int64_t t0,
                              int64_t t1, const double* Qx, const double* const* Qr, int64_t Q,
                              int A, const double* mu, int KT, uint16_t* xhi_h, float* xin_h,
                              unsigned* xnm_h, uint16_t* qhi_h, float* qn_h, void* xhi_d,
                              void* xin_d, void* xnm_d, void* qhi_d, void* qn_d, int chunks,
                              void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int64_t n_tiles = (N + 63) / 64;
  t0 = t0 < 0 ? 0 : (t0 > n_tiles ? n_tiles : t0);
  t1 = t1 < t0 ? t0 : (t1 > n_tiles ? n_tiles : t1);
  const int64_t W = (int64_t)KT * 32;  // bf16 per row / point
  static const bool dbg = getenv("DMLP_HOST_OPS_DEBUG") != nullptr;
  double tl[32];
  int nt = 0;
  auto now = [] {
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  const double t_start = dbg ? now() : 0.0;
  auto mark = [&] { if (dbg && nt < 32) tl[nt++] = now() - t_start; };
  chunks = chunks < 1 ? 1 : chunks;
  int rc = 0;
  float m = 0.0f;
  auto h2d = [&](void* d, const void* h, int64_t bytes) {
    if (bytes > 0 && dmlp::dma_copy(d, h, (size_t)bytes, st) != hipSuccess)  // (staging page-locked)
      rc |= 4;
  };
  for (int c = 0; c < chunks; ++c) {
    const int64_t a = t0 + (t1 - t0) * c / chunks, b = t0 + (t1 - t0) * (c + 1) / chunks;
    if (b <= a) continue;
    float mc = 0.0f;
    if (Xr ? dmlp_cpu_prep_data_tiles_rows(Xr, N, A, mu, KT, a, b, xhi_h, xin_h, &mc)
           : dmlp_cpu_prep_data_tiles(X, N, A, mu, KT, a, b, xhi_h, xin_h, &mc))
      rc |= 1;
    m = mc > m ? mc : m;
    mark();
    h2d((char*)xhi_d + (a - t0) * 64 * W * 2, xhi_h + a * 64 * W, (b - a) * 64 * W * 2);
    h2d((float*)xin_d + (a - t0) * 64, xin_h + a * 64, (b - a) * 64 * 4);
  }
  if (rc & 1) m = INFINITY;
  memcpy(xnm_h, &m, 4);
  if (xnm_d) h2d(xnm_d, xnm_h, 4);  // (null: the caller writes the word itself)
  for (int c = 0; c < chunks; ++c) {
    const int64_t q0 = Q * c / chunks, q1 = Q * (c + 1) / chunks;
    if (q1 <= q0) continue;
    if (Qr ? dmlp_cpu_prep_queries_rows(Qr + q0, q1 - q0, A, mu, KT, qhi_h + q0 * W, qn_h + q0)
           : dmlp_cpu_prep_queries(Qx + q0 * A, q1 - q0, A, mu, KT, qhi_h + q0 * W, qn_h + q0))
      rc |= 2;
    mark();
    h2d((char*)qhi_d + q0 * W * 2, qhi_h + q0 * W, (q1 - q0) * W * 2);
    h2d((float*)qn_d + q0, qn_h + q0, (q1 - q0) * 4);
  }
  mark();
  if (dbg) {
    fprintf(stderr, "[dmlp-hostops] threads %d tiles [%lld, %lld) us:", dmlp_host_threads(),
            (long long)t0, (long long)t1);
    for (int i = 0; i < nt; ++i) fprintf(stderr, " %.1f", tl[i]);
    fprintf(stderr, "\n");
  }
  return rc;
}

extern "C" int dmlp_host_ops_h2d_tiles(const double* X, int64_t N, int64_t t0, int64_t t1,
                                       const double* Qx, int64_t Q, int A, const double* mu,
                                       int KT, uint16_t* xhi_h, float* xin_h, unsigned* xnm_h,
                                       uint16_t* qhi_h, float* qn_h, void* xhi_d, void* xin_d,
                                       void* xnm_d, void* qhi_d, void* qn_d, int chunks,
                                       void* stream) {
  return host_ops_h2d_tiles(X, nullptr, N, t0, t1, Qx, nullptr, Q, A, mu, KT, xhi_h, xin_h, xnm_h,
                            qhi_h, qn_h, xhi_d, xin_d, xnm_d, qhi_d, qn_d, chunks, stream);
}
extern "C" int dmlp_host_ops_h2d_tiles_rows(const double* const* Xr, int64_t N, int64_t t0,
                                            int64_t t1, const double* const* Qr, int64_t Q, int A,
                                            const double* mu, int KT, uint16_t* xhi_h,
                                            float* xin_h, unsigned* xnm_h, uint16_t* qhi_h,
                                            float* qn_h, void* xhi_d, void* xin_d, void* xnm_d,
                                            void* qhi_d, void* qn_d, int chunks, void* stream) {
  return host_ops_h2d_tiles(nullptr, Xr, N, t0, t1, nullptr, Qr, Q, A, mu, KT, xhi_h, xin_h,
                            xnm_h, qhi_h, qn_h, xhi_d, xin_d, xnm_d, qhi_d, qn_d, chunks, stream);
}

// The whole image (tiles [0, n_tiles)).
extern "C" int dmlp_host_ops_h2d(const double* X, int64_t N, const double* Qx, int64_t Q, int A,
                                 const double* mu, int KT, uint16_t* xhi_h, float* xin_h,
                                 unsigned* xnm_h, uint16_t* qhi_h, float* qn_h, void* xhi_d,
                                 void* xin_d, void* xnm_d, void* qhi_d, void* qn_d, int chunks,
                                 void* stream) {
  return dmlp_host_ops_h2d_tiles(X, N, 0, (N + 63) / 64, Qx, Q, A, mu, KT, xhi_h, xin_h, xnm_h,
                                 qhi_h, qn_h, xhi_d, xin_d, xnm_d, qhi_d, qn_d, chunks, stream);
}

__global__ __launch_bounds__(256) void k_rows_from_i32(const int* __restrict__ src, int64_t n,
                                                      double* __restrict__ dst) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 4 <= n) {
    const int4 m = *(const int4*)(src + i);
    // IEEE division (correctly rounded, as the host's check): the exact input doubles
    *(double2*)(dst + i) = double2{(double)m.x / 1.0e6, (double)m.y / 1.0e6};
    *(double2*)(dst + i + 2) = double2{(double)m.z / 1.0e6, (double)m.w / 1.0e6};
  } else {
    for (int64_t j = i; j < n; ++j) dst[j] = (double)src[j] / 1.0e6;
  }
}

// fp64 rows from their lossless int32 form (host_prep.cpp dmlp_cpu_rows_i32): dst[i] = m / 1e6.
// src and dst 16-byte aligned.
extern "C" int dmlp_rows_from_i32(const int* src, int64_t n, double* dst, void* stream) {
  if (n <= 0) return 0;
  if (((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return -1;
  const int64_t blocks = (n + 1023) / 1024;
  hipLaunchKernelGGL(k_rows_from_i32, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     src, n, dst);
  DMLP_LAUNCH_CHECK();
  return 0;
}

extern "C" int dmlp_d2h_async(void* dst, const void* src, int64_t bytes, void* stream) {
  if (bytes <= 0) return 0;
  const hipError_t e = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost,
                                      (hipStream_t)stream);
  return e == hipSuccess ? 0 : -(int)e;
}

// ---------------------------------------------------------------- device render (dmlp_step)
// The single-term screen's fp16 operands rendered ON THE DEVICE from the rows that crossed PCIe
// for the exact re-rank anyway: lossless int32 m (x = m / 1e6, written out here as the fp64 rows
// the re-rank reads) or fp64.  The host then only packs int32 rows: no host render of the fp16
// image and query fragments, and 15 MB less over PCIe at the bench shape.  The arithmetic is
// host_prep.cpp's, bit for bit: c = x - mu in fp64, hi = fp16(fp32(c)) (round to nearest even,
// subnormals kept), |c|^2 as four fp64 partial sums s[a & 3] (each product and sum rounded) taken
// (s0 + s2) + (s1 + s3) and rounded to fp32.
//   mode 0 (dataset rows [r0, r0 + n), n padded to whole 64-point tiles; rows >= nvalid are
//          padding): the tile image (prep.hip's hi-only layout), xinit = -|c|^2 / 2 (-inf for
//          padding), the point-major copy xrow (the pair refine's member loads; may be null), and
//          the rounded-up max |c|^2 of these rows into *nmax (atomicMax of non-negative fp32 bits).
//   mode 1 (query rows): qhi [row][KT 32] and qn = |c|^2.
// A value with |c| >= 65504 (fp64 rows only: int32 rows are below 2^31 / 1e6 in magnitude) sets
// *bad.  done / rdy (nullable): the last workgroup to finish publishes *rdy = 1 with a release
// store — the early-start screen's ready word (screen_x1.hip k_screen_x1 rdy / qrdy).
// One-wave workgroups of <= 64 VGPRs: the kernel has to find wave slots beside an early-start
// screen, whose one-wave workgroups fill every CU (a multi-wave workgroup found none: every
// early wave timed out, profiles/r9e).
namespace {
template <int KT, bool I32>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) void k_render(
    const int* __restrict__ src32, const double* __restrict__ src64, int64_t r0, int64_t n,
    int64_t nvalid, int A, const double* __restrict__ mu, double* __restrict__ dst64, int mode,
    uint4* __restrict__ img, float* __restrict__ xq, uint4* __restrict__ xrow,
    unsigned* __restrict__ nmax, unsigned* __restrict__ bad, unsigned* __restrict__ done,
    unsigned* __restrict__ rdy) {
  constexpr int W = KT * 32;
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t p = r0 + i;
  const bool live = i < n;
  const bool valid = live && p < nvalid;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  bool ok = true;
  const int64_t t = p >> 6;
  const int pl = (int)(p & 63), rt = pl >> 4, r = pl & 15;
  for (int a0 = 0; a0 < W && live; a0 += 8) {
    unsigned hw[4];
#pragma unroll
    for (int j2 = 0; j2 < 4; ++j2) {
      unsigned short h2[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int a = a0 + 2 * j2 + e;
        double c = 0.0;
        if (valid && a < A) {
          double x;
          if (I32) {
            x = (double)src32[p * A + a] / 1.0e6;  // IEEE division: the exact input double
            if (dst64) dst64[p * A + a] = x;  // (null: the refine reads the int32 rows)
          } else {
            x = src64[p * A + a];
          }
          c = __dsub_rn(x, mu[a]);
          if (!(fabs(c) < 65504.0)) {
            ok = false;
            c = 0.0;
          }
          s[a & 3] = __dadd_rn(s[a & 3], __dmul_rn(c, c));
        }
        h2[e] = __builtin_bit_cast(unsigned short, (_Float16)(float)c);
      }
      hw[j2] = (unsigned)h2[0] | ((unsigned)h2[1] << 16);
    }
    const uint4 v = {hw[0], hw[1], hw[2], hw[3]};
    if (mode == 0) {
      const int kt = a0 >> 5, kg = (a0 >> 3) & 3;
      img[((t * 4 + rt) * KT + kt) * 64 + kg * 16 + r] = v;
      if (xrow) xrow[p * (W / 8) + (a0 >> 3)] = v;
    } else {
      img[p * (W / 8) + (a0 >> 3)] = v;
    }
  }
  const float ssf = (float)__dadd_rn(__dadd_rn(s[0], s[2]), __dadd_rn(s[1], s[3]));
  if (live) {
    if (mode == 0) xq[p] = valid ? -0.5f * ssf : -INFINITY;
    else xq[p] = ssf;
  }
  if (mode == 0 && nmax) {
    float up = valid ? __fadd_rn(__fmul_rn(ssf, 1.0f + 1.0e-6f), 1.0e-30f) : 0.0f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) up = fmaxf(up, __shfl_xor(up, o));
    if ((threadIdx.x & 63) == 0 && up > 0.0f) atomicMax(nmax, __float_as_uint(up));
  }
  if (!ok && bad) atomicOr(bad, 1u);
  if (done) {
    __builtin_amdgcn_wave_barrier();
    if (threadIdx.x == 0) {
      __threadfence();  // this workgroup's stores (and its atomics) before its count
      const unsigned prev = atomicAdd(done, 1u);
      if (prev == gridDim.x - 1 && rdy) {
        __threadfence();
        __hip_atomic_store(rdy, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

}  // namespace

extern "C" int dmlp_render_rows(int KT, int A, const int* src32, const double* src64, int64_t r0,
                                int64_t n, int64_t nvalid, const double* mu, double* dst64,
                                int mode, void* img, float* xq, void* xrow, unsigned* nmax,
                                unsigned* bad, unsigned* done, unsigned* rdy, void* stream) {
  if (n <= 0) {
    return 0;
  }
  if ((!src32 && !src64) || A < 1 || A > KT * 32 || !img || !xq ||
      (mode != 0 && mode != 1) || (mode == 0 && ((r0 & 63) || (n & 63))))
    return -1;
  const dim3 grid((unsigned)((n + 63) / 64)), block(64);
  hipStream_t st = (hipStream_t)stream;
#define DMLP_RENDER(KTV)                                                                       \
  do {                                                                                         \
    if (src32)                                                                                 \
      hipLaunchKernelGGL((k_render<KTV, true>), grid, block, 0, st, src32, nullptr, r0, n, nvalid, \
                         A, mu, dst64, mode, (uint4*)img, xq, (uint4*)xrow, nmax, bad, done, rdy); \
    else                                                                                       \
      hipLaunchKernelGGL((k_render<KTV, false>), grid, block, 0, st, nullptr, src64, r0, n,     \
                         nvalid, A, mu, dst64, mode, (uint4*)img, xq, (uint4*)xrow, nmax, bad,  \
                         done, rdy);                                                           \
  } while (0)
  if (KT == 1) DMLP_RENDER(1);
  else if (KT == 2) DMLP_RENDER(2);
  else if (KT == 4) DMLP_RENDER(4);
  else if (KT == 8) DMLP_RENDER(8);
  else return -1;
#undef DMLP_RENDER
  DMLP_LAUNCH_CHECK();
  return 0;
}

