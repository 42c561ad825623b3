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
#include <limits.h>

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
        if (V) V[o] = (int)pi;
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


// ---------------------------------------------------------------- radix-select path (k <= KSEL)
// One workgroup per row.  Keys are the distance bit patterns (non-negative doubles order like
// their u64 bits).  MSB-first 8-bit radix passes over the row, starting at the highest bit in
// which the row's min and max keys differ, narrow the k-th key's prefix until the rows at or
// below the prefix fit the LDS sort (<= KSEL entries); those are collected, bitonic-sorted in
// LDS under (dist asc, id desc) and the first k written out.  If exact ties at the k-th
// distance overflow KSEL, the entries strictly below it are taken plus the needed number of
// tied entries with the LARGEST ids (rows are stored in descending id order, so that is an
// ordered scan from the row start).  Per row: ~3-4 streaming passes instead of a full sort.
constexpr int KSEL = 2048;
constexpr int SEL_T = 256;

__device__ __forceinline__ int block_excl_scan(int v, int* tmp /*[SEL_T/64]*/, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) tmp[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int j = 0; j < SEL_T / 64; ++j) {
    const int t = tmp[j];
    if (j < w) base += t;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

__global__ __launch_bounds__(SEL_T) void k_select(const double* __restrict__ D, int64_t N,
                                                  const int* __restrict__ qidx,
                                                  const int* __restrict__ qk, int nb,
                                                  double* __restrict__ out_d,
                                                  int* __restrict__ out_i, int kstride) {
  __shared__ unsigned hist[SEL_T / 64][256];
  __shared__ double sd[KSEL];
  __shared__ int si[KSEL];
  __shared__ int scan_tmp[SEL_T / 64];
  __shared__ int s_sel, s_below, s_eq, s_cnt;
  __shared__ unsigned long long s_min, s_max;
  const int i = blockIdx.x;
  if (i >= nb) return;
  const int tid = threadIdx.x, w = tid >> 6;
  const int q = qidx[i];
  int k = qk[q];
  if ((int64_t)k > N) k = (int)N;
  if (k <= 0 || k > KSEL) return;
  const unsigned long long* row = (const unsigned long long*)(D + (int64_t)i * N);
  const int n = (int)N;

  // highest bit in which min and max key differ: no pass is wasted on the shared exponent
  unsigned long long mn = ~0ull, mx = 0;
  for (int j = tid; j < n; j += SEL_T) {
    const unsigned long long key = row[j];
    mn = key < mn ? key : mn;
    mx = key > mx ? key : mx;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if (tid == 0) { s_min = ~0ull; s_max = 0; }
  __syncthreads();
  if ((tid & 63) == 0) { atomicMin(&s_min, mn); atomicMax(&s_max, mx); }
  __syncthreads();
  const unsigned long long diff = s_min ^ s_max;
  // top = number of leading bits shared by every key; passes cover bits [shift, shift+8)
  int shift = diff ? 64 - __clzll((long long)diff) : 0;  // bits below `shift` still undecided
  unsigned long long prefix = s_min & (shift >= 64 ? 0ull : (~0ull << shift));
  int krem = k;   // entries still needed from the keys matching the prefix
  int cl = 0;     // entries whose key is strictly below the prefix range
  int ce = n;     // entries matching the prefix
  while (shift > 0 && cl + ce > KSEL) {
    const int sh = shift >= 8 ? shift - 8 : 0;
    const int width = shift - sh;
    for (int b = tid; b < (SEL_T / 64) * 256; b += SEL_T) (&hist[0][0])[b] = 0;
    __syncthreads();
    const unsigned long long hi_mask = shift >= 64 ? 0ull : (~0ull << shift);
    for (int j = tid; j < n; j += SEL_T) {
      const unsigned long long key = row[j];
      if ((key & hi_mask) == prefix)
        atomicAdd(&hist[w][(unsigned)(key >> sh) & ((1u << width) - 1)], 1u);
    }
    __syncthreads();
    int c = 0;
#pragma unroll
    for (int ww = 0; ww < SEL_T / 64; ++ww) c += (int)hist[ww][tid];
    int tot;
    const int ex = block_excl_scan(c, scan_tmp, &tot);
    if (ex < krem && krem <= ex + c) { s_sel = tid; s_below = ex; s_eq = c; }
    __syncthreads();
    prefix |= (unsigned long long)s_sel << sh;
    cl += s_below;
    krem -= s_below;
    ce = s_eq;
    shift = sh;
    __syncthreads();
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  const unsigned long long hi_mask = shift >= 64 ? 0ull : (~0ull << shift);
  int M;
  if (cl + ce <= KSEL) {
    // every key whose top bits are <= the prefix
    for (int j = tid; j < n; j += SEL_T) {
      const unsigned long long key = row[j];
      if ((key & hi_mask) <= prefix) {
        const int pos = atomicAdd(&s_cnt, 1);
        sd[pos] = __longlong_as_double((long long)key);
        si[pos] = n - 1 - j;
      }
    }
    __syncthreads();
    M = s_cnt;
  } else {
    // shift == 0: prefix is the exact k-th key T; cl < k keys below it, krem ties needed
    for (int j = tid; j < n; j += SEL_T) {
      const unsigned long long key = row[j];
      if (key < prefix) {
        const int pos = atomicAdd(&s_cnt, 1);
        sd[pos] = __longlong_as_double((long long)key);
        si[pos] = n - 1 - j;
      }
    }
    __syncthreads();
    int taken = 0;
    for (int j0 = 0; j0 < n && taken < krem; j0 += SEL_T) {  // ids descending
      const int j = j0 + tid;
      const bool eq = j < n && row[j] == prefix;
      int tot;
      const int ex = block_excl_scan(eq ? 1 : 0, scan_tmp, &tot);
      if (eq && taken + ex < krem) {
        sd[cl + taken + ex] = __longlong_as_double((long long)prefix);
        si[cl + taken + ex] = n - 1 - j;
      }
      taken += tot;
    }
    __syncthreads();
    M = k;
  }
  // bitonic sort of the M collected entries (padded to a power of two) in LDS
  int P = 1;
  while (P < M) P <<= 1;
  for (int j = M + tid; j < P; j += SEL_T) { sd[j] = INFINITY; si[j] = INT_MIN; }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < P / 2; t += SEL_T) {
        const int a = 2 * t - (t & (stride - 1));
        const int b = a + stride;
        const bool asc = (a & size) == 0;
        const double da = sd[a], db = sd[b];
        const int ia = si[a], ib = si[b];
        const bool sw = asc ? dmlp::key_less(db, ib, da, ia) : dmlp::key_less(da, ia, db, ib);
        if (sw) { sd[a] = db; sd[b] = da; si[a] = ib; si[b] = ia; }
      }
      __syncthreads();
    }
  }
  for (int j = tid; j < k; j += SEL_T) {
    out_d[(int64_t)q * kstride + j] = sd[j];
    out_i[(int64_t)q * kstride + j] = si[j];
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

extern "C" int dmlp_fallback_select_kmax(void) { return KSEL; }

extern "C" int64_t dmlp_fallback_select_bytes(int nb, int64_t N) {
  return (int64_t)align_up((size_t)nb * (size_t)N * 8);
}

// Exact top-k (k <= dmlp_fallback_select_kmax()) of queries qidx[0..nb) by radix select;
// workspace = dmlp_fallback_select_bytes(nb, N).  Rows with larger k are skipped.
extern "C" int dmlp_fallback_select(const double* X, int64_t N, int A, const double* Qx,
                                    const int* qidx, const int* qk, int nb, void* ws,
                                    int64_t ws_bytes, double* out_d, int* out_i, int kstride,
                                    void* stream) {
  if (nb <= 0 || N <= 0) return 0;
  if (N > 0x7fffffff) return -1;
  if (ws_bytes < dmlp_fallback_select_bytes(nb, N)) return -3;
  hipStream_t st = (hipStream_t)stream;
  double* D0 = (double*)ws;
  hipLaunchKernelGGL(k_rows_rev, dim3((unsigned)((N + 63) / 64), (unsigned)((nb + 63) / 64)),
                     dim3(256), 0, st, X, N, A, Qx, qidx, nb, D0, (int*)nullptr);
  DMLP_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_select, dim3((unsigned)nb), dim3(SEL_T), 0, st, D0, N, qidx, qk, nb,
                     out_d, out_i, kstride);
  DMLP_LAUNCH_CHECK();
  return 0;
}

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
