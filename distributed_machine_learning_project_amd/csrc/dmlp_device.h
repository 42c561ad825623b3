// dmlp_device.h — device-side building blocks shared by the CDNA4 kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DMLP_FNV_OFFSET 1469598103934665603ULL
#define DMLP_FNV_PRIME 1099511628211ULL

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) int i32x2;

namespace dmlp {

// Host <-> device copy through the SDMA engines whatever its size.  This runtime runs a
// hipMemcpyAsync below ~32 KiB (and every device-to-device copy) as a blit KERNEL
// (__amd_rocclr_copyBuffer): a wave slot beside the step's spinning screen and an engine switch
// in the stream.  The "no compute units" kind takes the DMA path for page-locked host memory as
// well (profiles/r10a_copy_kind.txt: a 4-byte H2D / D2H as one SDMA copy).  Both host pointers
// must be page-locked (hipHostMalloc / hipHostRegister) or device memory.
inline hipError_t dma_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, s);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Compiler + wave-level ordering point for LDS traffic of one wave (ds ops of a wave execute
// in order; this only stops the compiler from moving them across).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Exact squared L2 distance, reference semantics (engine.cpp:12-18): left-to-right over the
// attributes, each subtraction, product and sum separately rounded (no contraction).
__device__ __forceinline__ double exact_dist(const double* __restrict__ q,
                                             const double* __restrict__ x, int A) {
  double s = 0.0;
  for (int a = 0; a < A; ++a) {
    const double d = __dsub_rn(q[a], x[a]);
    s = __dadd_rn(s, __dmul_rn(d, d));
  }
  return s;
}

// (dist asc, id desc) total order.
__device__ __forceinline__ bool key_less(double da, int ia, double db, int ib) {
  // no short circuit: in the unrolled rank loops a branch per term became per-iteration
  // control flow whose flags the compiler spilled to scratch
  return (da < db) | ((da == db) & (ia > ib));
}

// Bitonic sort of E*64 (dist,id) keys held E per lane (element index r*64 + lane), ascending
// in key_less order.  Fully unrolled; register-resident.
template <int E>
__device__ __forceinline__ void wave_sort_keys(double (&d)[E], int (&id)[E]) {
  const int lane = lane_id();
  constexpr int P = E * 64;
#pragma unroll
  for (int size = 2; size <= P; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 64) {
        const int rs = stride >> 6;
#pragma unroll
        for (int r = 0; r < E; ++r) {
          if ((r & rs) == 0) {
            const int r2 = r | rs;
            const bool asc = (((r << 6) | lane) & size) == 0;
            const bool sw = asc ? key_less(d[r2], id[r2], d[r], id[r])
                                : key_less(d[r], id[r], d[r2], id[r2]);
            if (sw) {
              const double td = d[r]; d[r] = d[r2]; d[r2] = td;
              const int ti = id[r]; id[r] = id[r2]; id[r2] = ti;
            }
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const double pd = __shfl_xor(d[r], stride);
          const int pi = __shfl_xor(id[r], stride);
          const bool lower = (lane & stride) == 0;
          const bool asc = (((r << 6) | lane) & size) == 0;
          const bool want_min = (lower == asc);
          const bool take = want_min ? key_less(pd, pi, d[r], id[r]) : key_less(d[r], id[r], pd, pi);
          if (take) { d[r] = pd; id[r] = pi; }
        }
      }
    }
  }
}

// Bitonic sort of E*64 floats, DESCENDING.
template <int E>
__device__ __forceinline__ void wave_sort_desc(float (&v)[E]) {
  const int lane = lane_id();
  constexpr int P = E * 64;
#pragma unroll
  for (int size = 2; size <= P; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 64) {
        const int rs = stride >> 6;
#pragma unroll
        for (int r = 0; r < E; ++r) {
          if ((r & rs) == 0) {
            const int r2 = r | rs;
            const bool desc = (((r << 6) | lane) & size) == 0;
            const float a = v[r], b = v[r2];
            v[r] = desc ? fmaxf(a, b) : fminf(a, b);
            v[r2] = desc ? fminf(a, b) : fmaxf(a, b);
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < E; ++r) {
          const float p = __shfl_xor(v[r], stride);
          const bool lower = (lane & stride) == 0;
          const bool desc = (((r << 6) | lane) & size) == 0;
          v[r] = (lower == desc) ? fmaxf(v[r], p) : fminf(v[r], p);
        }
      }
    }
  }
}

// Select element `idx` (wave-uniform) of a register-distributed array.
template <int E, typename T>
__device__ __forceinline__ T wave_pick(const T (&v)[E], int idx) {
  T x = v[0];
#pragma unroll
  for (int r = 1; r < E; ++r)
    if ((idx >> 6) == r) x = v[r];
  return __shfl(x, idx & 63);
}

// Histogram h[256] (LDS) of keys: the bin b holding the kk-th largest key, i.e.
// sum(h[b+1..255]) < kk <= sum(h[b..255]); `above` += sum(h[b+1..255]).  -1 if sum(h) < kk.
// One wave; lane L owns bins 255-4L .. 252-4L (top first).
__device__ __forceinline__ int wave_kth_bin(const int* h, int kk, int& above) {
  const int lane = threadIdx.x & 63;
  int c[4], s = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) { c[i] = h[255 - (4 * lane + i)]; s += c[i]; }
  int incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  const unsigned long long hit = __ballot(incl >= kk);
  if (!hit) return -1;
  const int F = __ffsll((long long)hit) - 1;
  int b = -1, acc = incl - s, ab = 0;
  if (lane == F) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (b < 0 && acc + c[i] >= kk) { b = 255 - (4 * lane + i); ab = acc; }
      acc += c[i];
    }
  }
  b = __shfl(b, F);
  above += __shfl(ab, F);
  return b;
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int lane = lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Majority vote over the labels of ids[0..k) (ids < 0 skipped), tie -> larger label, none -> -1
// (engine.cpp:319-332).  One wave.  `hist` is a per-wave LDS scratch of hist_cap ints used when
// the label range [label_lo, label_hi) is small; otherwise an O(k^2/64) count.  lab(i, id)
// returns the label of entry i (a gather from the label table, or labels carried in LDS).
template <class LabFn>
__device__ __forceinline__ int wave_vote_by(const int* ids, int k, LabFn lab, int label_lo,
                                            int label_hi, int* hist, int hist_cap) {
  const int lane = lane_id();
  long long best = -1;  // (count << 32) | (label ^ 0x80000000)
  const int range = label_hi - label_lo;
  if (range > 0 && range <= hist_cap) {
    for (int i = lane; i < range; i += 64) hist[i] = 0;
    wave_sync();
    for (int i = lane; i < k; i += 64) {
      const int id = ids[i];
      if (id >= 0) atomicAdd(&hist[lab(i, id) - label_lo], 1);
    }
    wave_sync();
    for (int i = lane; i < range; i += 64) {
      const int c = hist[i];
      if (c > 0) {
        const long long key =
            ((long long)c << 32) | (long long)((unsigned)(i + label_lo) ^ 0x80000000u);
        best = key > best ? key : best;
      }
    }
  } else {
    for (int i = lane; i < k; i += 64) {
      const int id = ids[i];
      if (id < 0) continue;
      const int li = lab(i, id);
      int c = 0;
      for (int j = 0; j < k; ++j) {
        const int jd = ids[j];
        c += (jd >= 0 && lab(j, jd) == li);
      }
      const long long key = ((long long)c << 32) | (long long)((unsigned)li ^ 0x80000000u);
      best = key > best ? key : best;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const long long o = __shfl_xor(best, off);
    best = o > best ? o : best;
  }
  wave_sync();
  if (best < 0) return -1;
  return (int)((unsigned)(best & 0xffffffffll) ^ 0x80000000u);
}

__device__ __forceinline__ int wave_vote(const int* ids, int k, const int* __restrict__ labels,
                                         int label_lo, int label_hi, int* hist, int hist_cap) {
  return wave_vote_by(ids, k, [&](int, int id) { return labels[id]; }, label_lo, label_hi, hist,
                      hist_cap);
}

__device__ __forceinline__ uint64_t fnv_checksum(int label, const int* ids, int k) {
  uint64_t h = DMLP_FNV_OFFSET;
  h ^= (uint64_t)(int64_t)label;
  h *= DMLP_FNV_PRIME;
  for (int i = 0; i < k; ++i) {
    h ^= (uint64_t)(int64_t)(ids[i] + 1);
    h *= DMLP_FNV_PRIME;
  }
  return h;
}

}  // namespace dmlp

#define DMLP_LAUNCH_CHECK()                                   \
  do {                                                        \
    hipError_t e__ = hipGetLastError();                       \
    if (e__ != hipSuccess) return -(int)e__;                  \
  } while (0)
