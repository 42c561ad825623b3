// screen_stream.hip — barrier-free streaming variant of the bf16x3 MFMA screen (see screen.hip
// for the numerics: score a = <q',x'> - |x'|^2/2 in fp32 from a 3-term bf16 split, per-query
// threshold h = a_k - 2*eps_q that only rises, exact re-rank in refine.hip).
//
// Why a second kernel: profiling the LDS-shared kernel (profiles/README.md) showed the per-tile
// workgroup barrier coupling 8 waves, so every candidate append / threshold compaction of one
// wave stalled the other seven, and each wave re-read the whole tile from LDS for only 16
// queries.  Here every wave is its own workgroup:
//   * it owns 16*CT queries (CT MFMA column tiles; 64 queries at CT=4) for the whole slice, so
//     each 1 KiB A-fragment fetched is used by CT x 3 MFMAs;
//   * the 64-point data tiles (fragment-native layout from prep.hip) stream straight from
//     L2/Infinity Cache into a 2-deep register ring (global_load_dwordx4, two tiles ahead) —
//     no LDS staging, no barrier, nothing couples the 4 waves of a CU;
//   * acc is double-buffered: the MFMAs of tile i are issued first, then the (VALU/LDS) candidate
//     epilogue of tile i-1 runs while the matrix pipe works through them;
//   * candidate buffers live in LDS: per column 4 sub-buffers of SUB entries, one per row-group
//     lane, so appends need no cross-lane coordination; a lane appends <= 4 entries per (column
//     tile, row tile) group, and the column is compacted (20-round ballot radix select of the
//     k-th score, then round-robin re-deal) as soon as one of its sub-buffers passes SUB-4.
// LDS = CT*64*(SUB+1)*8 B (34.8 KiB at CT=4, SUB=16): four waves (one per SIMD) per CU.
#include "dmlp.h"
#include "dmlp_device.h"
#include <float.h>

namespace {

int g_stream_mode = 0;  // profiling ablations, see dmlp_set_screen_mode

template <int KT, int CT, int SUB>
struct StreamCfg {
  static constexpr int CAP = 4 * SUB;
  static constexpr int QW = 16 * CT;              // queries per wave / workgroup
  static constexpr int FRAGS = 4 * KT * 2;        // 1 KiB fragments per tile
  static constexpr int LDS = CT * 64 * (SUB + 1) * 8;
  static_assert(CAP <= 64, "one buffered entry per lane in compaction");
};

template <int KT, int CT, int SUB>
__global__ __launch_bounds__(64, 1) void k_screen_stream(
    const u32x4* __restrict__ xfrag, const f32x4* __restrict__ xinit4, int n_tiles,
    const bf16x8* __restrict__ qhi, const bf16x8* __restrict__ qlo, const float* __restrict__ qn,
    const int* __restrict__ qidx, const int* __restrict__ qk, int nq,
    const unsigned* __restrict__ xnmax_bits, const unsigned* __restrict__ bad, float eps_rel,
    int S, int tiles_per_slice, int n_qblocks, int mode, int* __restrict__ cand_ids,
    int* __restrict__ cand_cnt) {
  using C = StreamCfg<KT, CT, SUB>;
  constexpr int CAP = C::CAP;
  extern __shared__ __attribute__((aligned(16))) i32x2 sbuf[];

  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const int kg = lane >> 4;

  // ---- block -> (query block, slice); XCD-aware when S % 8 == 0 (see screen.hip)
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
  const int pbase = qb * C::QW;

  if (*bad) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int p = pbase + ct * 16 + c;
      if (lane < 16 && p < nq) cand_cnt[(int64_t)p * S + s] = -1;
    }
    return;
  }
  const float xnmax = __uint_as_float(*xnmax_bits);

  // ---- per column tile: query fragments, threshold, k, eps, sub-buffer count
  bf16x8 bh[CT][KT], bl[CT][KT];
  float h[CT], eps[CT];
  int kq[CT], cnt[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int p = pbase + ct * 16 + c;
    const bool valid = p < nq;
    const int q = valid ? qidx[p] : 0;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      bh[ct][kt] = qhi[(q * KT + kt) * 4 + kg];
      bl[ct][kt] = qlo[(q * KT + kt) * 4 + kg];
    }
    eps[ct] = eps_rel * (qn[q] + xnmax);
    kq[ct] = valid ? qk[q] : 0;
    h[ct] = valid ? -FLT_MAX : INFINITY;
    cnt[ct] = 0;
  }
  // sub-buffer (ct, m, cc): 17-entry pitch keeps the 16 columns of a lane group on distinct banks
  auto sub_ptr = [&](int ct, int m, int cc) { return sbuf + ((ct * 4 + m) * 16 + cc) * (SUB + 1); };

  // ---- compaction of column cc of column tile CT_ (one buffered entry per lane)
#define DMLP_COMPACT(CT_, CC)                                                                   \
  do {                                                                                          \
    const int cc_ = (CC);                                                                       \
    const int nmine_ = __shfl(cnt[CT_], cc_ + 16 * kg);                                         \
    const bool ok_ = c < nmine_;                                                                \
    i32x2 e_ = ok_ ? sub_ptr(CT_, kg, cc_)[c] : (i32x2){__float_as_int(-INFINITY), -1};        \
    const int ntot_ = __popcll(__ballot(ok_));                                                  \
    const int kc_ = __shfl(kq[CT_], cc_);                                                       \
    if (ntot_ >= kc_) {                                                                         \
      const unsigned bits_ = (unsigned)e_.x;                                                    \
      const unsigned u_ = ok_ ? (bits_ ^ ((bits_ >> 31) ? 0xffffffffu : 0x80000000u)) : 0u;     \
      unsigned T_ = 0;                                                                          \
      for (int bit = 31; bit >= 12; --bit) {                                                    \
        const unsigned cand_ = T_ | (1u << bit);                                                \
        if (__popcll(__ballot(u_ >= cand_)) >= kc_) T_ = cand_;                                 \
      }                                                                                         \
      const float ak_ = __uint_as_float((T_ >> 31) ? (T_ ^ 0x80000000u) : ~T_);                 \
      const float hn_ = ak_ - 2.0f * __shfl(eps[CT_], cc_);                                     \
      if (c == cc_) h[CT_] = fmaxf(h[CT_], hn_);                                                \
    }                                                                                           \
    const float hc_ = __shfl(h[CT_], cc_);                                                      \
    const bool keep_ = ok_ && __int_as_float(e_.x) >= hc_;                                      \
    const unsigned long long km_ = __ballot(keep_);                                             \
    const int kept_ = __popcll(km_);                                                            \
    dmlp::wave_sync();                                                                          \
    if (keep_) {                                                                                \
      const int pos_ = __popcll(km_ & dmlp::lanemask_lt());                                     \
      sub_ptr(CT_, pos_ & 3, cc_)[pos_ >> 2] = e_;                                              \
    }                                                                                           \
    dmlp::wave_sync();                                                                          \
    if (c == cc_) cnt[CT_] = (kept_ + 3 - kg) >> 2;                                             \
    if (kept_ > 4 * (SUB - 4) && c == cc_) { h[CT_] = INFINITY; cnt[CT_] = -(1 << 28); }         \
  } while (0)

  // ---- candidate epilogue of one finished tile (acc of tile J)
#define DMLP_EPILOGUE(ACC, J)                                                                   \
  do {                                                                                          \
    const int idbase_ = (t0 + (J)) * 64 + kg * 4;                                               \
    float mct_[CT];                                                                             \
    bool any_ = false;                                                                          \
    _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                         \
      float m_ = -INFINITY;                                                                     \
      _Pragma("unroll") for (int rt = 0; rt < 4; ++rt) m_ = fmaxf(m_, fmaxf(fmaxf(ACC[ct][rt][0], \
          ACC[ct][rt][1]), fmaxf(ACC[ct][rt][2], ACC[ct][rt][3])));                              \
      mct_[ct] = m_;                                                                            \
      any_ |= m_ >= h[ct];                                                                      \
    }                                                                                           \
    if ((mode & 1) == 0 && __ballot(any_)) {                                                    \
      _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                       \
        if (!__ballot(mct_[ct] >= h[ct])) continue;                                             \
        _Pragma("unroll") for (int rt = 0; rt < 4; ++rt) {                                      \
          const float mr_ = fmaxf(fmaxf(ACC[ct][rt][0], ACC[ct][rt][1]),                        \
                                  fmaxf(ACC[ct][rt][2], ACC[ct][rt][3]));                        \
          if (!__ballot(mr_ >= h[ct])) continue;                                                \
          i32x2* mys_ = sub_ptr(ct, kg, c);                                                     \
          _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                       \
            if (ACC[ct][rt][j] >= h[ct]) {                                                      \
              mys_[cnt[ct]] = (i32x2){__float_as_int(ACC[ct][rt][j]), idbase_ + rt * 16 + j};   \
              ++cnt[ct];                                                                        \
            }                                                                                   \
          }                                                                                     \
          unsigned long long nm_ = __ballot(cnt[ct] > SUB - 4);                                 \
          unsigned cols_ = (unsigned)((nm_ | (nm_ >> 16) | (nm_ >> 32) | (nm_ >> 48)) & 0xffffull); \
          while (cols_) {                                                                       \
            const int cc2_ = __ffs(cols_) - 1;                                                  \
            cols_ &= cols_ - 1;                                                                 \
            DMLP_COMPACT(ct, cc2_);                                                             \
          }                                                                                     \
        }                                                                                       \
      }                                                                                         \
    }                                                                                           \
  } while (0)

  // ---- 2-deep register ring of tiles + double-buffered accumulators
  bf16x8 A[2][4][KT][2];
  f32x4 Xi[2][4];
  f32x4 acc[2][CT][4];
#define DMLP_LOAD(I, R)                                                                         \
  do {                                                                                          \
    const int t_ = t0 + ((I) < nt ? (I) : nt - 1);                                              \
    const u32x4* src_ = xfrag + (int64_t)t_ * (C::FRAGS * 64) + lane;                          \
    _Pragma("unroll") for (int rt = 0; rt < 4; ++rt) {                                          \
      _Pragma("unroll") for (int kt = 0; kt < KT; ++kt) {                                       \
        A[R][rt][kt][0] = __builtin_bit_cast(bf16x8, src_[((rt * KT + kt) * 2 + 0) * 64]);      \
        A[R][rt][kt][1] = __builtin_bit_cast(bf16x8, src_[((rt * KT + kt) * 2 + 1) * 64]);      \
      }                                                                                         \
      Xi[R][rt] = xinit4[(int64_t)t_ * 16 + rt * 4 + kg];                                        \
    }                                                                                           \
  } while (0)
#define DMLP_MFMA(R)                                                                            \
  do {                                                                                          \
    _Pragma("unroll") for (int ct = 0; ct < CT; ++ct)                                           \
      _Pragma("unroll") for (int rt = 0; rt < 4; ++rt) acc[R][ct][rt] = Xi[R][rt];              \
    if (!(mode & 2)) {                                                                          \
      _Pragma("unroll") for (int kt = 0; kt < KT; ++kt) {                                       \
        _Pragma("unroll") for (int ct = 0; ct < CT; ++ct)                                       \
          _Pragma("unroll") for (int rt = 0; rt < 4; ++rt)                                      \
            acc[R][ct][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][rt][kt][0], bh[ct][kt], \
                                                                     acc[R][ct][rt], 0, 0, 0);   \
        _Pragma("unroll") for (int ct = 0; ct < CT; ++ct)                                       \
          _Pragma("unroll") for (int rt = 0; rt < 4; ++rt)                                      \
            acc[R][ct][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][rt][kt][0], bl[ct][kt], \
                                                                     acc[R][ct][rt], 0, 0, 0);   \
        _Pragma("unroll") for (int ct = 0; ct < CT; ++ct)                                       \
          _Pragma("unroll") for (int rt = 0; rt < 4; ++rt)                                      \
            acc[R][ct][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[R][rt][kt][1], bh[ct][kt], \
                                                                     acc[R][ct][rt], 0, 0, 0);   \
      }                                                                                         \
    }                                                                                           \
  } while (0)

  if (nt > 0) {
    DMLP_LOAD(0, 0);
    DMLP_LOAD(1, 1);
    for (int i0 = 0; i0 < nt; i0 += 2) {
      // step i0 (ring slot 0), then step i0+1 (ring slot 1)
      DMLP_MFMA(0);
      if (!(mode & 4)) DMLP_LOAD(i0 + 2, 0);
      if (i0 > 0) DMLP_EPILOGUE(acc[1], i0 - 1);
      if (i0 + 1 < nt) {
        DMLP_MFMA(1);
        if (!(mode & 4)) DMLP_LOAD(i0 + 3, 1);
        DMLP_EPILOGUE(acc[0], i0);
      }
    }
    if ((nt - 1) & 1) DMLP_EPILOGUE(acc[1], nt - 1);
    else DMLP_EPILOGUE(acc[0], nt - 1);
  }
  if (mode & 1) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) asm volatile("" ::"v"(acc[0][ct][0]), "v"(acc[1][ct][0]));
  }

  // ---- write this slice's candidates (ids only)
  dmlp::wave_sync();
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    for (int cc = 0; cc < 16; ++cc) {
      const int pp = pbase + ct * 16 + cc;
      if (pp >= nq) break;
      int* out = cand_ids + ((int64_t)pp * S + s) * CAP;
      const int nmine = __shfl(cnt[ct], cc + 16 * kg);
      if (__shfl(cnt[ct], cc) < 0) {
        if (lane == 0) cand_cnt[(int64_t)pp * S + s] = -1;
        continue;
      }
      const bool ok = c < nmine;
      const i32x2 e = ok ? sub_ptr(ct, kg, cc)[c] : (i32x2){0, -1};
      const float hc = __shfl(h[ct], cc);
      const bool keep = ok && __int_as_float(e.x) >= hc;
      const unsigned long long m = __ballot(keep);
      if (keep) out[__popcll(m & dmlp::lanemask_lt())] = e.y;
      if (lane == 0) cand_cnt[(int64_t)pp * S + s] = __popcll(m);
    }
  }
#undef DMLP_LOAD
#undef DMLP_MFMA
#undef DMLP_EPILOGUE
#undef DMLP_COMPACT
}

template <int KT, int CT, int SUB>
int launch_stream(const void* xfrag, const float* xinit, int64_t n_tiles, const void* qhi,
                  const void* qlo, const float* qn, const int* qidx, const int* qk, int nq,
                  const unsigned* xnmax, const unsigned* bad, float eps_rel, int S,
                  int* cand_ids, int* cand_cnt, hipStream_t stream) {
  using C = StreamCfg<KT, CT, SUB>;
  const int n_qblocks = (nq + C::QW - 1) / C::QW;
  const int tps = (int)((n_tiles + S - 1) / S);
  const int64_t grid = (int64_t)n_qblocks * S;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL((k_screen_stream<KT, CT, SUB>), dim3((unsigned)grid), dim3(64), C::LDS,
                     stream, (const u32x4*)xfrag, (const f32x4*)xinit, (int)n_tiles,
                     (const bf16x8*)qhi, (const bf16x8*)qlo, qn, qidx, qk, nq, xnmax, bad,
                     eps_rel, S, tps, n_qblocks, g_stream_mode, cand_ids, cand_cnt);
  DMLP_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// Streaming screen for k <= 32 (cap 64) and A <= 64 (KT <= 2).  Queries per workgroup:
// 64 at KT = 1 (CT = 4), 32 at KT = 2 (CT = 2, register budget).
extern "C" int dmlp_screen_stream_qw(int KT) { return KT == 1 ? 64 : (KT == 2 ? 32 : 0); }
extern "C" int dmlp_screen_stream_cap(void) { return 64; }
extern "C" int dmlp_screen_stream_kmax(void) { return 32; }

extern "C" void dmlp_set_stream_mode(int mode) { g_stream_mode = mode; }

extern "C" int dmlp_screen_stream(int KT, const void* xfrag, const float* xinit, int64_t n_tiles,
                                  const void* qhi, const void* qlo, const float* qn,
                                  const int* qidx, const int* qk, int nq,
                                  const unsigned* xnmax_bits, const unsigned* bad, float eps_rel,
                                  int S, int* cand_ids, int* cand_cnt, void* stream) {
  if (nq <= 0) return 0;
  if (S < 1 || n_tiles < 0 || n_tiles > 0x7fffffff / 64) return -1;
  hipStream_t st = (hipStream_t)stream;
  if (KT == 1)
    return launch_stream<1, 4, 16>(xfrag, xinit, n_tiles, qhi, qlo, qn, qidx, qk, nq, xnmax_bits,
                                   bad, eps_rel, S, cand_ids, cand_cnt, st);
  if (KT == 2)
    return launch_stream<2, 2, 16>(xfrag, xinit, n_tiles, qhi, qlo, qn, qidx, qk, nq, xnmax_bits,
                                   bad, eps_rel, S, cand_ids, cand_cnt, st);
  return -2;
}
