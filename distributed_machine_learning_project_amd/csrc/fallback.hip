// fallback.hip — exact top-k for the queries the screen does not take: k beyond the screen's
// capacity (k > 128), pathological ties (a candidate buffer overflowed), or data outside the
// screen's fp32 range.  Exact fp64 distance rows (reference order, no FMA) are written in
// DESCENDING id order, then a stable segmented radix sort (rocPRIM via hipCUB) orders each row by
// distance: stability keeps equal distances in descending id, i.e. exactly the reference's
// (dist asc, id desc) order without a 96-bit key.  The first k of each
// row are copied out.  Rare path; the workspace comes from the caller (no allocation here, so
// the call can be captured in a graph).
#include <hipcub/hipcub.hpp>

#include "dmlp.h"
#include "dmlp_device.h"

namespace {

// D[i][N-1-n] = exact dist(Qx[qidx[i]], X[n]); V[i][j] = N-1-j
__global__ __launch_bounds__(256) void k_rows_rev(const double* __restrict__ X, int64_t N, int A,
                                                  const double* __restrict__ Qx,
                                                  const int* __restrict__ qidx, int nb,
                                                  double* __restrict__ D, int* __restrict__ V) {
  constexpr int AC = 16;
  __shared__ double Qs[64][AC + 1];
  __shared__ double Xs[64][AC + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t pt0 = (int64_t)blockIdx.x * 64;
  const int qt0 = blockIdx.y * 64;
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  for (int a0 = 0; a0 < A; a0 += AC) {
    const int ac = A - a0 < AC ? A - a0 : AC;
    for (int e = tid; e < 64 * AC; e += 256) {
      const int r = e / AC, a = e % AC;
      const int qi = qt0 + r;
      Qs[r][a] = (qi < nb && a < ac) ? Qx[(int64_t)qidx[qi] * A + a0 + a] : 0.0;
      const int64_t pi = pt0 + r;
      Xs[r][a] = (pi < N && a < ac) ? X[pi * A + a0 + a] : 0.0;
    }
    __syncthreads();
    for (int a = 0; a < ac; ++a) {
      double qv[4], xv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) qv[i] = Qs[ty + 16 * i][a];
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[j] = Xs[tx + 16 * j][a];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const double dd = __dsub_rn(qv[i], xv[j]);
          acc[i][j] = __dadd_rn(acc[i][j], __dmul_rn(dd, dd));
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qi = qt0 + ty + 16 * i;
    if (qi >= nb) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t pi = pt0 + tx + 16 * j;
      if (pi < N) {
        const int64_t o = (int64_t)qi * N + (N - 1 - pi);
        D[o] = acc[i][j];
        V[o] = (int)pi;
      }
    }
  }
}

__global__ void k_seg_offsets(int* __restrict__ off, int nb, int64_t N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= nb) off[i] = (int)(i * N);
}

__global__ void k_take_k(const double* __restrict__ Ds, const int* __restrict__ Vs, int64_t N,
                         const int* __restrict__ qidx, const int* __restrict__ qk, int nb,
                         double* __restrict__ out_d, int* __restrict__ out_i, int kstride) {
  const int i = blockIdx.y;
  if (i >= nb) return;
  const int q = qidx[i];
  int k = qk[q];
  if (k > N) k = (int)N;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < k; j += gridDim.x * blockDim.x) {
    out_d[(int64_t)q * kstride + j] = Ds[(int64_t)i * N + j];
    out_i[(int64_t)q * kstride + j] = Vs[(int64_t)i * N + j];
  }
}

size_t sort_temp_bytes(int nb, int64_t N) {
  size_t bytes = 0;
  hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, bytes, (const double*)nullptr,
                                              (double*)nullptr, (const int*)nullptr, (int*)nullptr,
                                              (int)(nb * N), nb, (const int*)nullptr,
                                              (const int*)nullptr);
  return bytes;
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// Workspace bytes for nb rows of N points.
extern "C" int64_t dmlp_fallback_bytes(int nb, int64_t N) {
  const size_t items = (size_t)nb * (size_t)N;
  return (int64_t)(align_up(items * 8) * 2 + align_up(items * 4) * 2 + align_up((nb + 1) * 4) +
                   align_up(sort_temp_bytes(nb, N)));
}

// Exact top-k of queries qidx[0..nb) (k from qk[qidx[i]], clamped to N), written sorted to
// out_*[q*kstride + j].  nb * N must fit in int32 (callers chunk).
extern "C" int dmlp_fallback_topk(const double* X, int64_t N, int A, const double* Qx,
                                  const int* qidx, const int* qk, int nb, void* ws,
                                  int64_t ws_bytes, double* out_d, int* out_i, int kstride,
                                  void* stream) {
  if (nb <= 0 || N <= 0) return 0;
  if ((int64_t)nb * N > 0x7fffffff) return -1;
  if (ws_bytes < dmlp_fallback_bytes(nb, N)) return -3;
  hipStream_t st = (hipStream_t)stream;
  const size_t items = (size_t)nb * (size_t)N;
  char* p = (char*)ws;
  double* D0 = (double*)p; p += align_up(items * 8);
  double* D1 = (double*)p; p += align_up(items * 8);
  int* V0 = (int*)p; p += align_up(items * 4);
  int* V1 = (int*)p; p += align_up(items * 4);
  int* off = (int*)p; p += align_up((nb + 1) * 4);
  void* tmp = p;
  size_t tmp_bytes = sort_temp_bytes(nb, N);
  hipLaunchKernelGGL(k_rows_rev, dim3((unsigned)((N + 63) / 64), (unsigned)((nb + 63) / 64)),
                     dim3(256), 0, st, X, N, A, Qx, qidx, nb, D0, V0);
  DMLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_seg_offsets, dim3((nb + 256) / 256), dim3(256), 0, st, off, nb, N);
  DMLP_LAUNCH_CHECK();
  // non-negative doubles order like their bit patterns; stable LSD radix keeps id-desc ties
  hipError_t e = hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tmp_bytes, D0, D1, V0, V1,
                                                             (int)items, nb, off, off + 1, 0, 64, st);
  if (e != hipSuccess) return -(int)e;
  const int maxk_blocks = 64;
  hipLaunchKernelGGL(k_take_k, dim3(maxk_blocks, nb), dim3(256), 0, st, D1, V1, N, qidx, qk, nb,
                     out_d, out_i, kstride);
  DMLP_LAUNCH_CHECK();
  return 0;
}
