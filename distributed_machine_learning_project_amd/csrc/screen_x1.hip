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

// The pair epilogue (k_screen_x1 PAIR): every 16-entry screen, and the 32-entry one up to
// KT = DMLP_X1_PAIR32_KTMAX (1) — at KT >= 2 its 8-row groups cost the k in (32, 64] refine more
// (4-8 fragments per member) than the screen saves (profiles/r12r_pair32_kt_ab.txt)
#ifndef DMLP_X1_PAIR32_KTMAX
#define DMLP_X1_PAIR32_KTMAX 1
#endif
__host__ __device__ constexpr bool x1_pair(bool collect, int KT, int SUB) {
  return !collect && (SUB == 16 || KT <= DMLP_X1_PAIR32_KTMAX);
}

template <int KT, int SUB, int DEPTH, int CHECK>
struct X1Cfg {
  static constexpr int CT = 4;                  // MFMA column tiles per wave
  static constexpr int NCOL = 16 * CT;          // queries per wave (= workgroup)
  // column pitch in entries: 4 interleaved sub-buffers + 4 pad slots (which hold the 4
  // sub-buffer counts during a compaction); CP = 4 (mod 8) puts the 64 lanes of an append (16
  // columns x 4 sub-buffers, same fill) on 64 distinct banks
  static constexpr int CP = 4 * SUB + 4;
  // the fill check runs every CHECK steps, so a sub-buffer is compacted once it holds more than
  // SUB - CHECK entries (CHECK more appends always fit) and keeps at most SUB - CHECK of them
  static constexpr int CAPE = 4 * (SUB - CHECK);  // group entries a column may keep
  // group-id stride per (query, slice): the k class's (x1_sub: 16 or 32)
  static constexpr int IDCAP = 4 * ((SUB <= 16 ? 16 : 32) - 1);
  static constexpr int SBUF = NCOL * CP * 4;
  // a 512-byte ring of two 4-step windows of the rows' -|x'|^2/2 (the MFMA C operand), read with
  // ds_read_b128 instead of a 16-byte-per-lane buffer load per step
  static constexpr int XRING = 512;
  static constexpr int LDS = SBUF + XRING;
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

template <int KT, int SUB, int DEPTH, int CHECK, bool COLLECT, bool F16>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu((SUB == 32 || KT >= 4) ? 1 : 2))) void k_screen_x1(
    const u32x4* __restrict__ xfrag, const f32x4* __restrict__ xinit4, int n_tiles, int n_points,
    const bf16x8* __restrict__ qhi, const float* __restrict__ qn, const int* __restrict__ qidx,
    const int* __restrict__ qk, int nq, const unsigned* __restrict__ xnmax_bits,
    const unsigned* __restrict__ bad, float r1, float r2, float r3, int S, int s_first, int S_l,
    int tiles_per_slice, int n_qblocks, int hl, int* __restrict__ cand_ids,
    int* __restrict__ cand_cnt, float* __restrict__ cand_h, const float* __restrict__ hseed,
    int ccap, const unsigned* __restrict__ rdy, int rdy_tiles, int rdy_n,
    unsigned* __restrict__ estats, long long rdy_to) {
  // COLLECT (large k, second pass): the threshold is fixed at the query's seed hseed[p] (a
  // lower bound on its k-th best score - 2 eps from the first pass); a full buffer is flushed to
  // the column's global list (up to ccap group entries per (query, slice)) instead of compacted
  using C = X1Cfg<KT, SUB, DEPTH, CHECK>;
  // PAIR (not COLLECT; x1_pair): the hit test and the append run once per PAIR of steps, on the
  // 8-row group max (rows 4 kg .. 4 kg + 3 of both steps; entry index = pair * 4 + kg), instead of
  // per step on 4-row groups: the per-step max stays, the compare, the branch and the taken
  // step's append VALU halve (the screen is VALU-issue-bound: ~8.6 VALU per MFMA).  The
  // refine expands each entry to its 8 members (dmlp_screen_x1_group_rows).
  constexpr bool PAIR = x1_pair(COLLECT, KT, SUB);
  static_assert(!PAIR || (CHECK == 2 && DEPTH == 4), "the pair epilogue assumes 2-step checks");
  constexpr int CT = C::CT;
  constexpr int D = C::D;
  constexpr int NH = C::NCOL / 64;  // columns per lane in the lane-owns-column phases
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned* const sbuf = (unsigned*)smem;  // [col][CP] interleaved entries
  constexpr unsigned sb0 = 0u;             // its LDS byte offset

  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const int kg = lane >> 4;

  // ---- block -> (query block, slice) of this launch's S_l slices [s_first, s_first + S_l) of the
  // S the candidate lists are laid out for; XCD-aware when S_l % 8 == 0 (slice s stays on one
  // XCD's L2)
  const int b = blockIdx.x;
  int qb, s;
  if ((S_l & 7) == 0) {
    const int xcd = b & 7, local = b >> 3, m = S_l >> 3;
    const int sl = local / n_qblocks;
    qb = local - sl * n_qblocks;
    s = xcd * m + sl;
  } else {
    s = b % S_l;
    qb = b / S_l;
  }
  s += s_first;
  const int t0 = s * tiles_per_slice;
  int t1 = t0 + tiles_per_slice;
  if (t1 > n_tiles) t1 = n_tiles;
  const int nt = t1 > t0 ? t1 - t0 : 0;
  const int nsteps = nt * 4;
  const int pbase = qb * C::NCOL;

  if (*bad) {
    for (int col = lane; col < C::NCOL; col += 64)
      if (pbase + col < nq) cand_cnt[(int64_t)(pbase + col) * S + s] = -1;
    return;
  }
  // EARLY START (rdy != nullptr, S == 1): the data image is still crossing PCIe in rdy_n slices
  // of rdy_tiles tiles; rdy[i] turns nonzero once slice i landed, and its value is the slice's
  // max norm (fp32 bits, never 0: a slice of norm 0 publishes the smallest denormal — one copy
  // per slice carries both, profiles/r10a_step_copies.txt).  The wave waits for a slice before its
  // ring loads reach it, and a column's eps only covers the slices scanned so far: it grows at
  // each new slice (and its threshold drops by twice the growth), so every compaction's bound
  // holds for the entries it judges.  A wait that times out (rdy_to ticks of the constant-rate
  // wall clock, a few ms) marks the wave's queries overflowed (the pipeline escalates them).  The
  // ready word is written by a host-initiated DMA copy: it is polled with relaxed system-scope
  // loads and followed by a system-scope acquire fence before any image load.  Per wave: waits
  // that had to spin, eps growths and timeouts go to estats[0..2] at the end (the pipeline
  // reports them).
  int have = 0;  // slices known landed (wave-uniform)
  bool rdy_fail = false;
  unsigned n_wait = 0, n_grow = 0, n_to = 0;
  auto rdy_word = [&](int i) -> unsigned {
    unsigned* const f = const_cast<unsigned*>(rdy + i);
    return (unsigned)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  };
  auto wait_slice = [&](int i) -> bool {
    if (rdy_word(i) != 0u) return true;
    ++n_wait;
    const long long w0 = wall_clock64();
    for (;;) {
      __builtin_amdgcn_s_sleep(2);
      if (rdy_word(i) != 0u) return true;
      if (wall_clock64() - w0 > rdy_to) {
        ++n_to;
        return false;
      }
    }
  };
  // m folded with the max norms of slices [lo, hi] (system-scope loads: ~1-2 us each, so the
  // words of slices already seen are not read again)
  auto fold_xnm = [&](float m, int lo, int hi) {
    for (int i = lo; i <= hi; ++i) m = fmaxf(m, __uint_as_float(rdy_word(i)));
    return m;
  };
  // Once the last slice's word is set every slice has landed (the copies and their words run in
  // slice order on one stream): a wave that sees it takes the rest of the image at once instead
  // of probing slice by slice — each probe is a system-scope round trip on the wave's critical
  // path (the per-slice probes cost the screen ~0.075 ms: profiles/r7n_refine_ab.txt, r7s)
  auto widen = [&](int need) { return need < rdy_n - 1 && rdy_word(rdy_n - 1) != 0u ? rdy_n - 1 : need; };

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

  float xnmax;
  if (rdy) {
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
      // resolve these LDS loads here, not at the next use: otherwise the waitcnt pass sees them
      // pending after the conditional call and drains lgkmcnt at every following step
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    }
  };

  // ---- D-deep register ring of step fragments + double-buffered accumulators
  bf16x8 A[D][KT];
  f32x4 Xi[D];
  f32x4 acc[2][CT];
  float pm[CT];  // PAIR: the pair's first step's 4-row maxima
#define DMLP_LOADA(J, R)                                                                        \
  do {                                                                                          \
    _Pragma("unroll") for (int kt = 0; kt < KT; ++kt)                                           \
      A[R][kt] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(              \
          xr, lane * 16 + kt * ks, (J) * (KT * ks), 0));                                        \
  } while (0)
#define DMLP_LOADX(J, R)                                                                        \
  do {                                                                                          \
    Xi[R] = *(__attribute__((address_space(3))) const f32x4*)(size_t)(                          \
        xrb + (((J) >> 2) & 1) * 256 + ((J) & 3) * 64 + kg * 16);                               \
  } while (0)
#define DMLP_LOAD(J, R)                                                                         \
  do {                                                                                          \
    DMLP_LOADA(J, R);                                                                           \
    DMLP_LOADX(J, R);                                                                           \
  } while (0)
#define DMLP_MFMA(R, AB)                                                                        \
  do {                                                                                          \
    _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                         \
      acc[AB][ct] = mfma16<F16>(A[R][0], bh[ct][0], Xi[R]);                                     \
      _Pragma("unroll") for (int kt = 1; kt < KT; ++kt)                                         \
        acc[AB][ct] = mfma16<F16>(A[R][kt], bh[ct][kt], acc[AB][ct]);                           \
    }                                                                                           \
  } while (0)
#define DMLP_EPILOGUE(AB, J, ODD)                                                               \
  do {                                                                                          \
    /* per column tile: the 4-row group max (PAIR: on the pair's second step, the 8-row max), \
       and the wave's hit mask straight from the compare (an SGPR pair: the uniform branch    \
       below tests it with one s_cmp) */                                                       \
    float m_[CT];                                                                               \
    unsigned long long any_ = 0;                                                                \
    const bool first_ = PAIR && !(ODD); /* (ODD: J's parity, known at compile time) */          \
    _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                         \
      /* linear chains: the combiner makes 2 v_max3 of the pair's second step (pm + 4 rows) */ \
      if (PAIR && !first_)                                                                      \
        m_[ct] = fmaxf(fmaxf(fmaxf(fmaxf(pm[ct], acc[AB][ct][0]), acc[AB][ct][1]),              \
                             acc[AB][ct][2]), acc[AB][ct][3]);                                  \
      else                                                                                      \
        m_[ct] = fmaxf(fmaxf(fmaxf(acc[AB][ct][0], acc[AB][ct][1]), acc[AB][ct][2]),            \
                       acc[AB][ct][3]);                                                         \
      if (first_) pm[ct] = m_[ct];                                                              \
      else any_ |= __builtin_amdgcn_ballot_w64(m_[ct] >= h[ct]);                                \
    }                                                                                           \
    if (!first_ && (C::D == 4 || (J) < nsteps) && any_) {                                       \
      unsigned gl_ = PAIR ? (unsigned)(((J) >> 1) * 4 + kg) : (unsigned)((J) * 4 + kg);        \
      asm volatile("" : "+v"(gl_)); /* one VGPR: each key is a single v_and_or / v_bfi */       \
      /* branch-free: every lane writes its entry to the next free slot and advances only on  \
         a hit (slot cnt <= SUB-1 exists; a miss is overwritten later and never read) */       \
      _Pragma("unroll") for (int ct = 0; ct < CT; ++ct) {                                       \
        *(__attribute__((address_space(3))) unsigned*)(size_t)addr[ct] =                       \
            (__float_as_uint(m_[ct]) & 0xffff0000u) | gl_;                                      \
        addr[ct] += m_[ct] >= h[ct] ? 16u : 0u;                                                 \
      }                                                                                         \
    }                                                                                           \
  } while (0)
  // one compaction call site per CHECK steps (each inlined copy is ~8 KiB of code: one per
  // step of the unrolled ring would not stay in the instruction cache)
#define DMLP_CHECK()                                                                            \
  do {                                                                                          \
    /* the fill test at the check point itself (addresses only grow between checks): one    \
       compare per column tile every CHECK steps instead of one per tile per taken step */   \
    unsigned long long trig = 0;                                                                \
    _Pragma("unroll") for (int ct = 0; ct < CT; ++ct)                                           \
      trig |= __builtin_amdgcn_ballot_w64(addr[ct] > lim[ct]);                                  \
    if (trig) compact(false);                                                                   \
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
    pull_h();
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
    *(__attribute__((address_space(3))) float*)(size_t)(xrb + lane * 4) = xwin(0);
    xw = xwin(1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the ring reads stay after it
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
        const int j = j0 + r;  // D = 4: j < nsteps (nsteps % 4 == 0)
        DMLP_MFMA(r, r & 1);
        if (r == 0) {
          // window j0/4 + 1 (steps j0 + 4 .. j0 + 7) into the slot window j0/4 - 1 used (every
          // read of it is done: those steps were loaded into the register ring already)
          *(__attribute__((address_space(3))) float*)(size_t)(
              xrb + (((j0 >> 2) + 1) & 1) * 256 + lane * 4) = xw;
          xw = xwin((j0 >> 2) + 2);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
        DMLP_LOAD(j + D, r);
        if (j > 0) DMLP_EPILOGUE((r + 1) & 1, j - 1, (r + 1) & 1);
        // (PAIR: the appends come at even r — the pairs end at odd steps — and CHECK = 2 puts a
        // check one step behind each)
        if (r % CHECK == CHECK - 1) DMLP_CHECK();
      }
    }
    // the last issued step (padded up to a multiple of D)
    const int jl = ((nsteps + D - 1) / D) * D - 1;
    DMLP_EPILOGUE(jl & 1, jl, 1);  // (jl is odd: nsteps % 4 == 0)
  }
#undef DMLP_LOAD
#undef DMLP_LOADA
#undef DMLP_LOADX
#undef DMLP_MFMA
#undef DMLP_EPILOGUE
#undef DMLP_CHECK
  // final threshold over everything buffered, then the candidate ids
  compact(true);
  if (rdy && estats && lane == 0 && (n_wait | n_grow | n_to)) {
    atomicAdd(estats + 0, n_wait);
    atomicAdd(estats + 1, n_grow);
    atomicAdd(estats + 2, n_to);
  }
}

// the k class served by the SUB = 16 variant (two waves per SIMD, the pair epilogue): k <= 32,
// the pair refine's limit (its 56 kept group entries per column hold 32 groups + the 2 eps band:
// k = 32 at the bench shape 3.49 -> 2.40 ms, k 1-32 3.27 -> 2.20, no escalation,
// profiles/r11t_sub16_ab.txt); DMLP_X1_SUB16_KMAX narrows it (16: the SUB = 32 variant from k 17)
int x1_sub16_kmax() {
  static const int v = [] {
    const char* e = getenv("DMLP_X1_SUB16_KMAX");
    const int k = e && *e ? atoi(e) : 32;
    return k < 1 ? 32 : k > 32 ? 32 : k;
  }();
  return v;
}
// The same class boundary at every KT.  (KT 2's 16-entry screen leaves the early start's copies
// no wave slot, and with the pair epilogue on the 32-entry screen KT 2 once ran k in (16, 32]
// faster there with the early start (r11z); with that epilogue at KT 1 only (x1_pair) the 16-entry
// screen wins: A = 48 / 64, k = 32, 3.98-4.64 vs 4.45-4.88 ms, profiles/r12w_kt2_sub_ab.txt.)
int x1_sub(int KT, int kmax) {
  (void)KT;
  return kmax <= x1_sub16_kmax() ? 16 : 32;
}

// One launch over slices [s_first, s_first + S_l) of an S-slice split (cand_* laid out for S).
// (Variants measured slower and deleted — the LDS-ring screen, 8 column tiles per wave, the
// per-tile / exec-masked appends, the query-block early start: profiles/README.md, r9*.)
template <int KT, int SUB, int DEPTH, int CHECK, bool F16>
int launch_x1(int hl, const void* xfrag, const float* xinit, int64_t n_tiles, int64_t n_points,
              const void* qhi, const float* qn, const int* qidx, const int* qk, int nq,
              const unsigned* xnmax, const unsigned* bad, float r1, float r2, float r3, int S,
              int s_first, int S_l, int* cand_ids, int* cand_cnt, float* cand_h,
              hipStream_t stream, const float* hseed = nullptr, int ccap = 0,
              const unsigned* rdy = nullptr, int rdy_tiles = 1, int rdy_n = 0,
              unsigned* estats = nullptr, long long rdy_to = 0) {
  using C = X1Cfg<KT, SUB, DEPTH, CHECK>;
  const int n_qblocks = (nq + C::NCOL - 1) / C::NCOL;  // workgroups per slice
  const int tps = (int)((n_tiles + S - 1) / S);
  const int64_t grid = (int64_t)n_qblocks * S_l;
  if (grid <= 0) return 0;
#define DMLP_X1_LAUNCH(COLL)                                                                    \
  hipLaunchKernelGGL((k_screen_x1<KT, SUB, DEPTH, CHECK, COLL, F16>), dim3((unsigned)grid),     \
                     dim3(64), C::LDS, stream, (const u32x4*)xfrag, (const f32x4*)xinit,        \
                     (int)n_tiles, (int)n_points, (const bf16x8*)qhi, qn, qidx, qk, nq, xnmax,  \
                     bad, r1, r2, r3, S, s_first, S_l, tps, n_qblocks, hl, cand_ids, cand_cnt,  \
                     cand_h, hseed, ccap, rdy, rdy_tiles, rdy_n, estats, rdy_to)
  if (hseed) {  // the COLLECT pass (SUB = 16, fp16 only: see dmlp_screen_x1_collect)
    if constexpr (SUB == 16 && F16) DMLP_X1_LAUNCH(true);
    else return -3;
  } else {
    DMLP_X1_LAUNCH(false);
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
  (void)kmax;
  return x1_kt_ok(KT) ? 64 : 0;
}
// group ids per (query, slice) (refine expands each to its dmlp_screen_x1_group_rows members)
extern "C" int dmlp_screen_x1_cap_kt(int KT, int kmax) { return 4 * (x1_sub(KT, kmax) - 1); }
extern "C" int dmlp_screen_x1_cap(int kmax) { return dmlp_screen_x1_cap_kt(1, kmax); }
// rows per group entry of the screen that serves (KT, kmax) (and of its early-start form): 8 (the
// pair epilogue, x1_pair: steps 2p and 2p + 1, rows 4 kg .. 4 kg + 3 of each) or 4 (consecutive
// rows); the COLLECT pass always 4
extern "C" int dmlp_screen_x1_group_rows_kt(int KT, int kmax) {
  return x1_pair(false, KT, x1_sub(KT, kmax)) ? 8 : 4;
}
extern "C" int dmlp_screen_x1_group_rows(int kmax) { return dmlp_screen_x1_group_rows_kt(1, kmax); }
// resident workgroups (= waves) per CU: LDS-bound at 17.5 KiB (SUB 16, 4 tiles) / 33.5 KiB
// (SUB 32); the 8-tile variant runs one wave per SIMD (register-bound)
extern "C" int dmlp_screen_x1_waves_per_cu(int kmax) {
  return x1_sub(1, kmax) == 16 ? 8 : 4;
}
// the same for an image of KT fragments per step: A > 64 (KT = 4, 8) runs one wave per SIMD (the
// query and ring fragments take the registers of two)
extern "C" int dmlp_screen_x1_waves_per_cu_kt(int KT, int kmax) {
  return KT >= 4 ? 4 : x1_sub(KT, kmax) == 16 ? 8 : 4;
}
// a slice must stay below 2^16 4-row groups (16-bit group index in an entry)
extern "C" int64_t dmlp_screen_x1_min_slices(int64_t n_tiles) { return (n_tiles + 4095) / 4096; }

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
  return launch_x1<KTV, 16, 4, 2, true>(1, xfrag, xinit, n_tiles, n_points, qhi, qn, qidx, qk,  \
                                       nq, xnmax_bits, bad, r1, r2, r3, S, 0, S, cand_ids,      \
                                       cand_cnt, cand_h, st, hseed, ccap)
  if (KT == 1) DMLP_X1C(1);
  if (KT == 2) DMLP_X1C(2);
  if (KT == 4) DMLP_X1C(4);
  DMLP_X1C(8);
#undef DMLP_X1C
}

// Slices [s_first, s_first + S_l) of an S-slice screen (cand_* laid out for all S slices): a
// caller streaming the dataset in chunks screens each chunk's slices as soon as it landed.
extern "C" int dmlp_screen_x1_part(int KT, int hl, int A, const void* xfrag, const float* xinit,
                                   int64_t n_tiles, int64_t n_points, const void* qhi,
                                   const float* qn, const int* qidx, const int* qk, int nq,
                                   int kmax, const unsigned* xnmax_bits, const unsigned* bad,
                                   int S, int s_first, int S_l, int* cand_ids, int* cand_cnt,
                                   float* cand_h, void* stream) {
  if (nq <= 0 || S_l <= 0) return 0;
  if (S < 1 || s_first < 0 || s_first + S_l > S || n_tiles < 0 || n_tiles > 0x7fffffff / 64 ||
      n_points > n_tiles * 64)
    return -1;
  if ((n_tiles + S - 1) / S > 4096) return -4;  // 16-bit group index per slice
  if (kmax > 64 || !x1_kt_ok(KT) || A > KT * 32) return -3;
  if (hl != 1 && hl != 2) return -1;
  float r1, r2, r3;
  dmlp_screen_x1_bound2(A, hl, &r1, &r2, &r3);
  hipStream_t st = (hipStream_t)stream;
#define DMLP_X1_ARGS hl, xfrag, xinit, n_tiles, n_points, qhi, qn, qidx, qk, nq, xnmax_bits, bad, r1, \
                     r2, r3, S, s_first, S_l, cand_ids, cand_cnt, cand_h, st
  const bool s32 = x1_sub(KT, kmax) == 32;
  // hl = 1: the host's fp16 image + fp16 query fragments; hl = 2: prep.hip's bf16 hi/lo image
#define DMLP_X1_PICK(F16)                                                                      \
  do {                                                                                         \
    if (KT == 1) return s32 ? launch_x1<1, 32, 4, 2, F16>(DMLP_X1_ARGS)                        \
                            : launch_x1<1, 16, 4, 2, F16>(DMLP_X1_ARGS);                       \
    if (KT == 2) return s32 ? launch_x1<2, 32, 4, 2, F16>(DMLP_X1_ARGS)                        \
                            : launch_x1<2, 16, 4, 2, F16>(DMLP_X1_ARGS);                       \
    if (KT == 4) return s32 ? launch_x1<4, 32, 4, 2, F16>(DMLP_X1_ARGS)                        \
                            : launch_x1<4, 16, 4, 2, F16>(DMLP_X1_ARGS);                       \
    return s32 ? launch_x1<8, 32, 4, 2, F16>(DMLP_X1_ARGS)                                     \
               : launch_x1<8, 16, 4, 2, F16>(DMLP_X1_ARGS);                                    \
  } while (0)
  if (hl == 1) DMLP_X1_PICK(true);
  DMLP_X1_PICK(false);
#undef DMLP_X1_PICK
#undef DMLP_X1_ARGS
}

extern "C" int dmlp_screen_x1(int KT, int hl, int A, const void* xfrag, const float* xinit,
                              int64_t n_tiles, int64_t n_points, const void* qhi, const float* qn,
                              const int* qidx, const int* qk, int nq, int kmax,
                              const unsigned* xnmax_bits, const unsigned* bad, int S,
                              int* cand_ids, int* cand_cnt, float* cand_h, void* stream) {
  return dmlp_screen_x1_part(KT, hl, A, xfrag, xinit, n_tiles, n_points, qhi, qn, qidx, qk, nq,
                             kmax, xnmax_bits, bad, S, 0, S, cand_ids, cand_cnt, cand_h, stream);
}

// The single-term screen over the host's fp16 image while that image is still crossing PCIe
// (pipeline.hip's early start): one data slice per workgroup (S = 1), rdy[i] != 0 once image
// tiles [i rdy_tiles, (i + 1) rdy_tiles) landed, its value the slice's max norm (fp32 bits).  The
// result is the one dmlp_screen_x1(KT, 1, ...) gives with S = 1 once every slice landed.
extern "C" int dmlp_screen_x1_early(int KT, int A, const void* xfrag, const float* xinit,
                                    int64_t n_tiles, int64_t n_points, const void* qhi,
                                    const float* qn, const int* qidx, const int* qk, int nq,
                                    int kmax, const unsigned* bad, const unsigned* rdy,
                                    int rdy_tiles, int rdy_n, int* cand_ids, int* cand_cnt,
                                    float* cand_h, unsigned* estats, void* stream) {
  if (nq <= 0) return 0;
  if (n_tiles < 1 || n_tiles > 4096 || n_points > n_tiles * 64 || !rdy || rdy_tiles < 1 ||
      rdy_n < 1 || (int64_t)rdy_tiles * rdy_n < n_tiles)
    return -1;
  if (kmax > 64 || !x1_kt_ok(KT) || A > KT * 32) return -3;
  float r1, r2, r3;
  dmlp_screen_x1_bound2(A, 1, &r1, &r2, &r3);
  hipStream_t st = (hipStream_t)stream;
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
  const bool s32 = x1_sub(KT, kmax) == 32;
#define DMLP_X1E(KTV, SUBV)                                                                     \
  return launch_x1<KTV, SUBV, 4, 2, true>(1, xfrag, xinit, n_tiles, n_points, qhi, qn, qidx,    \
                                         qk, nq, bad, bad, r1, r2, r3, 1, 0, 1, cand_ids,       \
                                         cand_cnt, cand_h, st, nullptr, 0, rdy, rdy_tiles,      \
                                         rdy_n, estats, rdy_to)
  if (KT == 1) { if (s32) DMLP_X1E(1, 32); DMLP_X1E(1, 16); }
  if (KT == 2) { if (s32) DMLP_X1E(2, 32); DMLP_X1E(2, 16); }
  if (KT == 4) { if (s32) DMLP_X1E(4, 32); DMLP_X1E(4, 16); }
  if (s32) DMLP_X1E(8, 32);
  DMLP_X1E(8, 16);
#undef DMLP_X1E
}
