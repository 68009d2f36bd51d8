// Causal AliBi multi-head attention, flash style (no T x T score matrix in HBM).
//
// Reference: MultiHeadAttention.forward (vap/modules.py:82-110), AliBi bias/mask
// (modules.py:169-202): score[h,i,j] = (q_i . k_j) * scale + m_h * j for j <= i, -inf above the
// diagonal; scale = 1/sqrt(dim) (quirk Q5).  Softmax is shift-invariant per row, so the kernel
// adds m_h * (j - i) (<= 0) instead of m_h * j: same probabilities, better conditioned in fp32.
//
// Work split: one workgroup = 64 queries of one (sequence, head); 4 waves x 16 queries.
// S^T = K Q^T on the MFMA (A = K tile from LDS, B = Q from registers) puts each query on a lane
// (col = lane & 15) so the online softmax is lane-local + 2 butterflies; O^T = V^T P^T takes P
// straight from registers as the B operand (no P round trip through LDS; the k order inside a
// k-step is permuted consistently on both operands).  V is staged transposed (V^T[d][key]).
#include <cstdlib>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

constexpr int QB = 64, KB = 64, HDIM = 64;

template <typename T>
struct AttnGeom {
  static constexpr int CE = 16 / sizeof(T);
  static constexpr int CPR = HDIM / CE;                // 16-B chunks per K row (8 bf16, 16 f32)
  static constexpr int KROW = HDIM * sizeof(T);        // 128 / 256 B
  static constexpr int VROW = KB * sizeof(T) + (sizeof(T) == 2 ? 8 : 16);  // padded V^T row
  static constexpr int KGD = HDIM / (4 * CE);          // k-groups over head dim (2 / 4)
  VAP_DEV static int kswz(int row, int c) { return sizeof(T) == 2 ? (c ^ ((row >> 1) & 7)) : (c ^ (row & 15)); }
};

template <typename T>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  using G = AttnGeom<T>;
  __shared__ __attribute__((aligned(16))) unsigned char sk[KB * G::KROW];
  __shared__ __attribute__((aligned(16))) unsigned char sv[HDIM * G::VROW];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int qb = blockIdx.x, h = blockIdx.y, s = blockIdx.z;
  const int ks = a.kv_swap ? (s ^ 1) : s;  // cross-attention: the other speaker of the same clip
  const T* Qs = (const T*)a.Q + (int64_t)s * a.q_seq + h * HDIM;
  const T* Ks = (const T*)a.K + (int64_t)ks * a.k_seq + h * HDIM;
  const T* Vs = (const T*)a.V + (int64_t)ks * a.v_seq + h * HDIM;
  const float slope = a.slopes[h];
  const int q = qb * QB + w * 16 + (lane & 15);
  const int qc = q < a.T ? q : a.T - 1;

  chunk16 qf[G::KGD];
#pragma unroll
  for (int kg = 0; kg < G::KGD; ++kg)
    qf[kg] = *(const chunk16*)(Qs + (int64_t)qc * a.q_ld + (kg * 4 + (lane >> 4)) * G::CE);

  float m = -INFINITY, lsum = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kb = 0; kb <= qb; ++kb) {
    const int key0 = kb * KB;
    // ---- stage K tile [key][d] (swizzled) and V^T tile [d][key]
    for (int i = tid; i < KB * G::CPR; i += 256) {
      const int row = i / G::CPR, c = i - row * G::CPR;
      const int key = key0 + row;
      chunk16 kv = {0, 0, 0, 0}, vv = {0, 0, 0, 0};
      if (key < a.T) {
        kv = *(const chunk16*)(Ks + (int64_t)key * a.k_ld + c * G::CE);
        vv = *(const chunk16*)(Vs + (int64_t)key * a.v_ld + c * G::CE);
      }
      *(chunk16*)(sk + row * G::KROW + G::kswz(row, c) * 16) = kv;
      const T* ve = (const T*)&vv;
#pragma unroll
      for (int e = 0; e < G::CE; ++e) *(T*)(sv + (c * G::CE + e) * G::VROW + row * sizeof(T)) = ve[e];
    }
    __syncthreads();

    // ---- S^T tiles: st[kt][r] = score(key = key0 + kt*16 + (lane>>4)*4 + r, query q)
    f32x4 st[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int row = kt * 16 + (lane & 15);
#pragma unroll
      for (int kg = 0; kg < G::KGD; ++kg) {
        const chunk16 kf = *(const chunk16*)(sk + row * G::KROW + G::kswz(row, kg * 4 + (lane >> 4)) * 16);
        acc = mfma_chunk<T>(kf, qf[kg], acc);
      }
      st[kt] = acc;
    }
    float bm = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = key0 + kt * 16 + (lane >> 4) * 4 + r;
        float v = st[kt][r] * a.scale + slope * (float)(key - q);
        if (key > q) v = -INFINITY;
        st[kt][r] = v;
        bm = fmaxf(bm, v);
      }
    bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
    bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
    const float mn = fmaxf(m, bm);
    const float alpha = expf(m - mn);
    m = mn;
    float ps = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = expf(st[kt][r] - mn);
        st[kt][r] = p;
        ps += p;
      }
    lsum = lsum * alpha + ps;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;

    // ---- O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const unsigned char* vrow = sv + (dt * 16 + (lane & 15)) * G::VROW;
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const u32x2 v0 = *(const u32x2*)(vrow + (32 * kk + (lane >> 4) * 4) * 2);
          const u32x2 v1 = *(const u32x2*)(vrow + (32 * kk + 16 + (lane >> 4) * 4) * 2);
          const chunk16 af = {v0.x, v0.y, v1.x, v1.y};
          bf16x8 pb = {(bf16)st[2 * kk][0], (bf16)st[2 * kk][1], (bf16)st[2 * kk][2], (bf16)st[2 * kk][3],
                       (bf16)st[2 * kk + 1][0], (bf16)st[2 * kk + 1][1], (bf16)st[2 * kk + 1][2],
                       (bf16)st[2 * kk + 1][3]};
          o[dt] = mfma_chunk<T>(af, __builtin_bit_cast(chunk16, pb), o[dt]);
        }
      } else {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          const f32x4 vv = *(const f32x4*)(vrow + (kt * 16 + (lane >> 4) * 4) * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[r], st[kt][r], o[dt], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  float lt = lsum + __shfl_xor(lsum, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  const float inv = 1.0f / lt;
  if (q < a.T) {
    T* orow = (T*)a.O + (int64_t)s * a.o_seq + (int64_t)q * a.o_ld + h * HDIM;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = dt * 16 + (lane >> 4) * 4;
      store4(orow + d, o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv);
    }
  }
}

// ------------------------------------------------------------------------------------------
// bf16 perf-mode attention: 128 queries per workgroup (4 waves x 32 = two 16-query MFMA column
// blocks per wave, sharing every K/V fragment read), K/V tiles of 64 keys double-buffered in LDS
// (register prefetch of tile kb+1 while tile kb computes), V kept row-major and fed to the
// O^T = V^T P^T MFMA through ds_read_b64_tr_b16 (hardware transpose read: no scalar transposed
// LDS writes), scores in the log2 domain (v_exp_f32), causal mask only on diagonal tiles and
// fully-masked tiles skipped per wave.
// ------------------------------------------------------------------------------------------
constexpr int QB2 = 128, KB2 = 64, TROW = 128;  // K / V tile rows: 64 bf16 = 128 B
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

VAP_DEV int kswz2(int row, int c) { return c ^ ((row >> 1) & 7); }

VAP_DEV u32x2 tr_read(const unsigned char* p) {
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)p);
  return __builtin_bit_cast(u32x2, v);
}

// ------------------------------------------------------------------------------------------
// attn4: the bf16 kernel.  Online softmax in the exp2 domain with the softmax VALU cut down (the
// kernel is VALU- and latency-bound at head_dim 64: ~256 MFMA FLOPs but ~4 VALU ops per score):
//  * the query term of the AliBi bias cancels in the softmax, so the score is s*c2 + sl2*key: the
//    S MFMA's C operand starts at the key bias of a 32-key tile (one register set); the tile and
//    32-key offsets go into the running max instead of the scores;
//  * lazy rescaling: the running max m is only raised (and O, l rescaled) when a tile's max exceeds
//    it by more than 8 (log2 domain), decided wave-uniformly; otherwise exp2(v - m) <= 256 is exact
//    enough for the bf16 P operand and the fp32 sums;
//  * v_mfma_f32_32x32x16_bf16 throughout (a 16x16x32 MFMA holds the SIMD's vector issue for 8 of its
//    16 cycles, a 32x32x16 for 8 of 32); the 32x32 layout puts 16 keys of ONE query in a lane
//    (column = query = lane & 31, rows = keys 8(r>>2) + 4h + (r&3), h = lane >> 5), so a query's max
//    over a 64-key tile is lane-local max3 steps and one v_permlane32_swap.
//   S^T (64 keys x 32 queries of a wave) = K Q'^T: 2 key tiles x 4 k-steps;
//   P^T feeds O^T = V^T P^T straight from the S registers (registers 8s .. 8s+7 of a key tile are
//     the B fragment of k-step s; its k order, keys 16s + 8(j>>2) + 4h + (j&3), is matched by the
//     two ds_read_b64_tr_b16 reads of the V^T fragment); a ones row-block gives the denominators
//     from the same bf16 P;
//   K image: ds_read_b128 rows, chunk ^ ((row>>1)&7); V image: transposed reads, chunk ^ 4((row>>1)&1)
//     (both conflict-free).
// Dispatch, XCD-aware: the dispatcher deals workgroups to the 8 XCDs round-robin, so block b runs
// on XCD b % 8.  When the (sequence, head) pairs divide by 8, XCD x takes the pairs p = x (mod 8),
// in groups of `grp` pairs whose q-blocks run longest-first within the group: the K/V of the pairs
// in flight (grp x <= 256 KiB) stay in that XCD's 4 MiB L2 instead of being fetched again for every
// q-block (FETCH_SIZE 319 -> 96 MB per 128-sequence launch; a longest-first order over all pairs
// puts one pair's q-blocks far apart in time).
// Measured and dropped: K / V tiles by LDS-DMA into a 3-slot ring two tiles ahead with the K
// fragments of a 32-key half read together (no faster: 149 vs 149 us per 128 x 1000 launch); a
// software pipeline across key tiles (S_j issued, then the previous tile's P.V, then tile j's softmax
// beside those MFMAs; V one tile behind K in LDS): 194 VGPRs, 2 waves per SIMD, 0.92 -> 1.03-1.09 ms
// per bench step (forced to 3 waves: 13 spilled VGPRs, 1.34 ms) -- the third wave per SIMD already
// hides the softmax behind another wave's MFMAs better than one wave's own pipeline.  Key tiles
// from the diagonal down with the tile max only on the wave's top two tiles (the diagonal tiles set
// the running max; the older tiles skip 15 v_max3 + the ballot): 153 -> 142 us on the 128 x 1000
// microbenchmark but no change in the bench (0.99 vs 1.00 ms per step), and a guard against exp2
// overflow (re-run on a non-finite row sum) spilled 18 VGPRs (1.6 ms): dropped.
// ------------------------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));
VAP_DEV f32x16 mfma32(chunk16 a, chunk16 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
VAP_DEV int vswz4(int row, int c) { return c ^ (((row >> 1) & 1) << 2); }
VAP_DEV float xmax2(float v) {  // max with lane ^ 32
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return fmaxf(a, b);
}

#ifndef ATT_DIAG
#define ATT_DIAG 0  // diagnostics (A/B builds only, outputs not meaningful): 1 no exp, 2 no row-sum MFMA, 4 K/V tile 0 only
#endif
__global__ __launch_bounds__(256, 3) void attn4_kernel(AttnArgs a, int nqb, int grp) {
  __shared__ __attribute__((aligned(16))) unsigned char kv[2][2][KB2 * TROW];  // [buf][K,V]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int npair = a.H * a.S;
  int hs, qb;
  if (grp > 0 && (npair & 7) == 0) {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, px = npair >> 3;  // pairs per XCD
    const int g = j / (grp * nqb), r = j - g * grp * nqb;
    const int gp = min(grp, px - g * grp);                                // pairs in this group
    const int lv = r / gp;
    qb = nqb - 1 - lv;
    hs = (g * grp + (r - lv * gp)) * 8 + x;
  } else {
    hs = blockIdx.x % npair;
    qb = nqb - 1 - (int)(blockIdx.x / npair);
  }
  const int h = hs % a.H, s = hs / a.H;
  const int ks = a.kv_swap ? (s ^ 1) : s;
  const bf16* Qs = (const bf16*)a.Q + (int64_t)s * a.q_seq + h * HDIM;
  const __amdgpu_buffer_rsrc_t rK = make_rsrc((const bf16*)a.K + (int64_t)ks * a.k_seq + h * HDIM, (uint32_t)a.T * a.k_ld * 2);
  const __amdgpu_buffer_rsrc_t rV = make_rsrc((const bf16*)a.V + (int64_t)ks * a.v_seq + h * HDIM, (uint32_t)a.T * a.v_ld * 2);
  constexpr float LOG2E = 1.4426950408889634f;
  constexpr float TAU = 8.0f;
  const float c2 = a.scale * LOG2E, sl2 = a.slopes[h] * LOG2E;
  const int qw0 = a.q0 + qb * QB2 + w * 32;  // first query of this wave
  const int qlast = min(a.q0 + qb * QB2 + QB2 - 1, a.T - 1);
  const int nkb = qlast / KB2 + 1;
  const int hl = lane >> 5, ql = lane & 31;
  const int qv = qw0 + ql;  // this lane's query

  // Q'^T fragments (B of the S MFMA): lane holds dims 16k + 8h .. +8 of its query, pre-scaled
  chunk16 qf[4];
  {
    const int qc = qv < a.T ? qv : a.T - 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bf16x8 q = *(const bf16x8*)(Qs + (int64_t)qc * a.q_ld + 16 * k + 8 * hl);
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = (bf16)((float)q[e] * c2);
      qf[k] = __builtin_bit_cast(chunk16, q);
    }
  }
  // key bias of the lane's S registers within a 32-key tile (the C operand of the S MFMA)
  f32x16 kb0;
#pragma unroll
  for (int r = 0; r < 16; ++r) kb0[r] = sl2 * (float)(8 * (r >> 2) + 4 * hl + (r & 3));
  const float off32 = sl2 * 32.0f, off64 = sl2 * (float)KB2;

  float m = -INFINITY;  // running max of the true log2 scores
  f32x16 o0 = {}, o1 = {}, ls = {};
  const bf16x8 ones8 = {(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f};
  const chunk16 ones = __builtin_bit_cast(chunk16, ones8);

  // staging: 2 K + 2 V chunks per thread, scalar tile offset
  const int srow = tid >> 3, sc = tid & 7;
  const uint32_t vkoff0 = (uint32_t)(srow * a.k_ld + sc * 8) * 2, vkoff1 = vkoff0 + 32u * a.k_ld * 2;
  const uint32_t vvoff0 = (uint32_t)(srow * a.v_ld + sc * 8) * 2, vvoff1 = vvoff0 + 32u * a.v_ld * 2;
  const uint32_t ktile = (uint32_t)KB2 * a.k_ld * 2, vtile = (uint32_t)KB2 * a.v_ld * 2;
  const int ldsK0 = srow * TROW + kswz2(srow, sc) * 16, ldsK1 = (srow + 32) * TROW + kswz2(srow + 32, sc) * 16;
  const int ldsV0 = srow * TROW + vswz4(srow, sc) * 16, ldsV1 = (srow + 32) * TROW + vswz4(srow + 32, sc) * 16;
  chunk16 rk[2], rv[2];
  auto gload = [&](int kb) {
    rk[0] = buf_load16(rK, vkoff0, kb * ktile);
    rk[1] = buf_load16(rK, vkoff1, kb * ktile);
    rv[0] = buf_load16(rV, vvoff0, kb * vtile);
    rv[1] = buf_load16(rV, vvoff1, kb * vtile);
  };
  auto lstore = [&](int buf) {
    *(chunk16*)(kv[buf][0] + ldsK0) = rk[0];
    *(chunk16*)(kv[buf][0] + ldsK1) = rk[1];
    *(chunk16*)(kv[buf][1] + ldsV0) = rv[0];
    *(chunk16*)(kv[buf][1] + ldsV1) = rv[1];
  };
  // K fragment of key tile t, k-step k: row 32t + ql, chunk 2k + hl (the 32t part is an immediate)
  int koff[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) koff[k] = ql * TROW + kswz2(ql, 2 * k + hl) * 16;
  // V^T fragment, dims 32u + ql, keys 32t + 16s + 4hl + {0..3} (+8 for elements 4..7): the lane
  // supplies row 4hl + q, columns 32u + 16(g&1) + 4p of its 16-lane group g (lane = 16g + 4q + p)
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = (lane >> 4) & 1;
  int voff[2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
    voff[u] = (4 * hl + tq) * TROW + vswz4(4 * hl + tq, 4 * u + 2 * tg + (tp >> 1)) * 16 + (tp & 1) * 8;

  auto tile = [&](int kb, auto cur_c) {
    constexpr int cur = (ATT_DIAG & 4) ? 0 : decltype(cur_c)::value;
    if (!(ATT_DIAG & 4) && kb + 1 < nkb) gload(kb + 1);
    const int key0 = kb * KB2;
    if (key0 <= qw0 + 31) {  // wave-uniform: some key of the tile is visible to some query of the wave
      const unsigned char* Kt = kv[cur][0];
      const unsigned char* Vt = kv[cur][1];
      f32x16 st[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        st[t] = kb0;
#pragma unroll
        for (int k = 0; k < 4; ++k) st[t] = mfma32(*(const chunk16*)(Kt + t * 32 * TROW + koff[k]), qf[k], st[t]);
      }
      if (key0 + KB2 - 1 > qw0) {  // wave-uniform: a diagonal tile
        // register (t, r) holds key key0 + 4 hl + 32t + 8(r>>2) + (r&3): one compare against an inline
        // constant per register
        const int dd = qv - key0 - 4 * hl;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (32 * t + 8 * (r >> 2) + (r & 3) > dd) st[t][r] = -INFINITY;
      }
      float b0 = st[0][0], b1 = st[1][0];
#pragma unroll
      for (int r = 1; r < 16; ++r) {
        b0 = fmaxf(b0, st[0][r]);
        b1 = fmaxf(b1, st[1][r]);
      }
      const float tofs = off64 * (float)kb;
      const float bm = xmax2(fmaxf(b0, b1 + off32)) + tofs;  // the tile's max true score of the lane's query
      if (__ballot(bm > m + TAU)) {  // wave-uniform: raise the running max, rescale O and the sums
        const float mn = fmaxf(m, bm);
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        m = mn;
        o0 *= alpha;
        o1 *= alpha;
        ls *= alpha;
      }
      const float m0 = m - tofs, m1 = m0 - off32;
      bf16x8 pb[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const float mt = t ? m1 : m0;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            pb[t][k][e] = (ATT_DIAG & 1) ? (bf16)(st[t][8 * k + e] - mt) : (bf16)__builtin_amdgcn_exp2f(st[t][8 * k + e] - mt);
        }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const chunk16 p = __builtin_bit_cast(chunk16, pb[t][k]);
          const int ro = (32 * t + 16 * k) * TROW;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const u32x2 v0 = tr_read(Vt + ro + voff[u]);
            const u32x2 v1 = tr_read(Vt + ro + 8 * TROW + voff[u]);
            const chunk16 vf = {v0.x, v0.y, v1.x, v1.y};
            if (u == 0) o0 = mfma32(vf, p, o0);
            else o1 = mfma32(vf, p, o1);
          }
          if (!(ATT_DIAG & 2)) ls = mfma32(ones, p, ls);
        }
    }
    if (!(ATT_DIAG & 4) && kb + 1 < nkb) lstore(cur ^ 1);
    if (!(ATT_DIAG & 4)) __syncthreads();
  };

  gload(0);
  lstore(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; kb += 2) {  // unrolled by 2: the LDS buffer index is a constant
    tile(kb, std::integral_constant<int, 0>{});
    if (kb + 1 < nkb) tile(kb + 1, std::integral_constant<int, 1>{});
  }
  // O^T: lane holds its query's dims 32u + 8g + 4hl + e in register 4g + e of o_u
  const float inv = 1.0f / ls[0];
  if (qv < a.T) {
    bf16* orow = (bf16*)a.O + (int64_t)s * a.o_seq + (int64_t)qv * a.o_ld + h * HDIM;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      store4(orow + 8 * g + 4 * hl, o0[4 * g] * inv, o0[4 * g + 1] * inv, o0[4 * g + 2] * inv, o0[4 * g + 3] * inv);
      store4(orow + 32 + 8 * g + 4 * hl, o1[4 * g] * inv, o1[4 * g + 1] * inv, o1[4 * g + 2] * inv, o1[4 * g + 3] * inv);
    }
  }
}

}  // namespace


// ------------------------------------------------------------------------------------------
// fp32 parity-mode attention on split-bf16 operands (the default of the fp32 mode; VAP_FP32_EXACT=1
// runs attn_kernel<float> above).  Same work split and softmax as attn_kernel (64 queries x one
// (sequence, head), 4 waves x 16 queries, S^T = K Q^T, O^T = V^T P^T with P from registers), but
// every fp32 operand x is carried as hi = bf16(x), lo = bf16(x - hi) and every product as
// hi hi + hi lo + lo hi: three v_mfma_f32_16x16x32_bf16 per 16x16x32 tile-step (48 cycles) instead
// of eight v_mfma_f32_16x16x4_f32 (256).  K and V are split once per workgroup as they are staged (K
// as two [key][d] images, V as two transposed [d][key] images); Q once per lane; P per key tile from
// the fp32 probabilities.  Scores live in the log2 domain (scale and slope pre-multiplied by log2 e):
// v_exp_f32 instead of libm expf.
// ------------------------------------------------------------------------------------------
namespace {
constexpr int SVROW = KB * 2 + 8;  // padded V^T row (bf16): 136 B
constexpr float LOG2E = 1.4426950408889634f;

VAP_DEV void split8(const f32x4& a, const f32x4& b, chunk16& hi, chunk16& lo) {
  const bf16x8 h = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
  const bf16x8 l = {(bf16)(a[0] - (float)h[0]), (bf16)(a[1] - (float)h[1]), (bf16)(a[2] - (float)h[2]),
                    (bf16)(a[3] - (float)h[3]), (bf16)(b[0] - (float)h[4]), (bf16)(b[1] - (float)h[5]),
                    (bf16)(b[2] - (float)h[6]), (bf16)(b[3] - (float)h[7])};
  hi = __builtin_bit_cast(chunk16, h);
  lo = __builtin_bit_cast(chunk16, l);
}

VAP_DEV f32x4 mfma3(const chunk16& ah, const chunk16& al, const chunk16& bh, const chunk16& bl, f32x4 acc) {
  acc = mfma_chunk<bf16>(ah, bl, acc);
  acc = mfma_chunk<bf16>(al, bh, acc);
  return mfma_chunk<bf16>(ah, bh, acc);
}

__global__ __launch_bounds__(256) void attn_split_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char skh[KB * 128], skl[KB * 128];      // K [key][d] hi / lo
  __shared__ __attribute__((aligned(16))) unsigned char svh[HDIM * SVROW], svl[HDIM * SVROW];  // V^T [d][key]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int qb = blockIdx.x, h = blockIdx.y, s = blockIdx.z;
  const int ks = a.kv_swap ? (s ^ 1) : s;
  const float* Qs = (const float*)a.Q + (int64_t)s * a.q_seq + h * HDIM;
  const float* Ks = (const float*)a.K + (int64_t)ks * a.k_seq + h * HDIM;
  const float* Vs = (const float*)a.V + (int64_t)ks * a.v_seq + h * HDIM;
  const float sc = a.scale * LOG2E, sl2 = a.slopes[h] * LOG2E;
  const int q = qb * QB + w * 16 + (lane & 15);
  const int qc = q < a.T ? q : a.T - 1;

  chunk16 qh[2], ql[2];  // d = 32kk + 8(lane>>4) .. +7 of query q
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const float* qr = Qs + (int64_t)qc * a.q_ld + kk * 32 + (lane >> 4) * 8;
    split8(*(const f32x4*)qr, *(const f32x4*)(qr + 4), qh[kk], ql[kk]);
  }

  float m = -INFINITY, lsum = 0.f;
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K / V of the next key block are loaded into registers while this one computes (buffer loads: keys
  // >= T read as zero); thread item it = tid + 256 i covers keys 2 (it >> 4) and +1, floats 4 (it & 15) .. +3,
  // so V^T takes one 4-byte write per (d, key pair) and K one 8-byte write per row and half
  const __amdgpu_buffer_rsrc_t rK = make_rsrc(Ks, (uint32_t)((int64_t)a.T * a.k_ld * 4));
  const __amdgpu_buffer_rsrc_t rV = make_rsrc(Vs, (uint32_t)((int64_t)a.T * a.v_ld * 4));
  f32x4 kr[2][2], vr[2][2];
  auto kvload = [&](int key0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int it = tid + 256 * i, key = key0 + 2 * (it >> 4), c = it & 15;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        kr[i][e] = __builtin_bit_cast(f32x4, buf_load16(rK, (uint32_t)(((int64_t)(key + e) * a.k_ld + c * 4) * 4), 0));
        vr[i][e] = __builtin_bit_cast(f32x4, buf_load16(rV, (uint32_t)(((int64_t)(key + e) * a.v_ld + c * 4) * 4), 0));
      }
    }
  };
  kvload(0);
  for (int kb = 0; kb <= qb; ++kb) {
    const int key0 = kb * KB;
    // ---- stage K hi / lo [key][d] (8-B halves of swizzled 16-B chunks) and V^T hi / lo [d][key]
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int it = tid + 256 * i, row = 2 * (it >> 4), c = it & 15;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const f32x4 kv = kr[i][e];
        const bf16x4 khi = {(bf16)kv[0], (bf16)kv[1], (bf16)kv[2], (bf16)kv[3]};
        const bf16x4 klo = {(bf16)(kv[0] - (float)khi[0]), (bf16)(kv[1] - (float)khi[1]),
                            (bf16)(kv[2] - (float)khi[2]), (bf16)(kv[3] - (float)khi[3])};
        const int off = (row + e) * 128 + kswz2(row + e, c >> 1) * 16 + (c & 1) * 8;
        *(bf16x4*)(skh + off) = khi;
        *(bf16x4*)(skl + off) = klo;
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const float v0 = vr[i][0][d], v1 = vr[i][1][d];
        const bf16 h0 = (bf16)v0, h1 = (bf16)v1;
        const bf16 l0 = (bf16)(v0 - (float)h0), l1 = (bf16)(v1 - (float)h1);
        typedef bf16 bf16x2 __attribute__((ext_vector_type(2)));
        *(bf16x2*)(svh + (c * 4 + d) * SVROW + row * 2) = bf16x2{h0, h1};
        *(bf16x2*)(svl + (c * 4 + d) * SVROW + row * 2) = bf16x2{l0, l1};
      }
    }
    __syncthreads();
    if (kb < qb) kvload(key0 + KB);  // the next block flies while this one computes

    // ---- S^T tiles: st[kt][r] = score (log2 domain) of key key0 + kt*16 + (lane>>4)*4 + r, query q
    f32x4 st[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int row = kt * 16 + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int off = row * 128 + kswz2(row, kk * 4 + (lane >> 4)) * 16;
        acc = mfma3(*(const chunk16*)(skh + off), *(const chunk16*)(skl + off), qh[kk], ql[kk], acc);
      }
      st[kt] = acc;
    }
    float bm = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = key0 + kt * 16 + (lane >> 4) * 4 + r;
        float v = st[kt][r] * sc + sl2 * (float)(key - q);
        if (key > q) v = -INFINITY;
        st[kt][r] = v;
        bm = fmaxf(bm, v);
      }
    bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
    bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
    const float mn = fmaxf(m, bm);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    float ps = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(st[kt][r] - mn);
        st[kt][r] = p;
        ps += p;
      }
    lsum = lsum * alpha + ps;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;

    // ---- O^T[d][q] += V^T[d][key] P^T[key][q]; keys of k-step kk in the order of the lanes' P registers
    chunk16 ph[2], pl[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) split8(st[2 * kk], st[2 * kk + 1], ph[kk], pl[kk]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int vr = (dt * 16 + (lane & 15)) * SVROW;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int k0 = (32 * kk + (lane >> 4) * 4) * 2, k1 = (32 * kk + 16 + (lane >> 4) * 4) * 2;
        const u32x2 h0 = *(const u32x2*)(svh + vr + k0), h1 = *(const u32x2*)(svh + vr + k1);
        const u32x2 l0 = *(const u32x2*)(svl + vr + k0), l1 = *(const u32x2*)(svl + vr + k1);
        o[dt] = mfma3(chunk16{h0.x, h0.y, h1.x, h1.y}, chunk16{l0.x, l0.y, l1.x, l1.y}, ph[kk], pl[kk], o[dt]);
      }
    }
    __syncthreads();
  }
  float lt = lsum + __shfl_xor(lsum, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  const float inv = 1.0f / lt;
  if (q < a.T) {
    float* orow = (float*)a.O + (int64_t)s * a.o_seq + (int64_t)q * a.o_ld + h * HDIM;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int d = dt * 16 + (lane >> 4) * 4;
      store4(orow + d, o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv);
    }
  }
}
}  // namespace

template <typename T>
hipError_t launch_attention(const AttnArgs& a, hipStream_t st) {
  if (a.T <= 0 || a.S <= 0 || a.H <= 0) return hipErrorInvalidValue;
  if constexpr (sizeof(T) == 2) {
    if (a.q0 < 0 || a.q0 >= a.T) return hipErrorInvalidValue;
    const int nqb = (a.T - a.q0 + QB2 - 1) / QB2;
    constexpr int grp = 8;  // (sequence, head) pairs per XCD group: K/V of 8 pairs x <= 256 KiB in L2
    hipLaunchKernelGGL(attn4_kernel, dim3(nqb * a.H * a.S), dim3(256), 0, st, a, nqb, grp);
    return hipGetLastError();
  }
  if (a.q0 != 0) return hipErrorInvalidValue;
  dim3 grid((a.T + QB - 1) / QB, a.H, a.S);
  if constexpr (sizeof(T) == 4) {
    if (a.split) {  // the fp32 parity mode's default: split-bf16 operands
      hipLaunchKernelGGL(attn_split_kernel, grid, dim3(256), 0, st, a);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((attn_kernel<T>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

template hipError_t launch_attention<float>(const AttnArgs&, hipStream_t);
template hipError_t launch_attention<bf16>(const AttnArgs&, hipStream_t);

// ------------------------------------------------------------------------------------------
// Attention weights (VapGPT.forward(attention=True), vap/model.py:264-267; the `att` the reference
// MultiHeadAttention returns, modules.py:96-110): softmax(q k^T * scale + m_h * j, causal) rows,
// materialised as P[s][h][i][j] (fp32, zeros above the diagonal).  A diagnostic path, not the hot
// one: one wave per query row, fp32 dot products from the layer's Q / K (fp32 or bf16 storage).
// The AliBi term uses m_h * (j - i), equal after the row softmax to the reference's m_h * j.
// ------------------------------------------------------------------------------------------
namespace {
template <typename T>
__global__ __launch_bounds__(256) void attn_probs_kernel(AttnArgs a, float* __restrict__ out, int64_t out_seq,
                                                         int64_t out_head) {
  __shared__ float qs[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 4 + w, h = blockIdx.y, s = blockIdx.z;
  if (i >= a.T) return;  // wave-uniform; no block-wide sync below
  const T* Q = (const T*)a.Q + (int64_t)s * a.q_seq + (int64_t)i * a.q_ld + h * 64;
  const int skv = a.kv_swap ? (s ^ 1) : s;
  const T* K = (const T*)a.K + (int64_t)skv * a.k_seq + h * 64;
  qs[w][lane] = to_f32(Q[lane]) * a.scale;
  __builtin_amdgcn_wave_barrier();
  const float m = a.slopes[h];
  float* o = out + (int64_t)s * out_seq + (int64_t)h * out_head + (int64_t)i * a.T;
  // pass 1: scores of keys j = lane + 64 t (j <= i) -> row max
  float mx = -INFINITY;
  for (int j = lane; j <= i; j += 64) {
    const T* k = K + (int64_t)j * a.k_ld;
    float d = 0.f;
#pragma unroll 16
    for (int c = 0; c < 64; ++c) d = fmaf(qs[w][c], to_f32(k[c]), d);
    const float v = d + m * (float)(j - i);
    o[j] = v;  // scratch: the raw score, rewritten below
    mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j <= i; j += 64) {
    const float e = __expf(o[j] - mx);
    o[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  const float inv = 1.0f / sum;
  for (int j = lane; j < a.T; j += 64) o[j] = j <= i ? o[j] * inv : 0.f;
}
}  // namespace

template <typename T>
hipError_t launch_attn_probs(const AttnArgs& a, float* out, int64_t out_seq, int64_t out_head, hipStream_t st) {
  if (a.T <= 0 || a.S <= 0 || a.H <= 0 || !out) return hipErrorInvalidValue;
  hipLaunchKernelGGL((attn_probs_kernel<T>), dim3((a.T + 3) / 4, a.H, a.S), dim3(256), 0, st, a, out, out_seq, out_head);
  return hipGetLastError();
}
template hipError_t launch_attn_probs<float>(const AttnArgs&, float*, int64_t, int64_t, hipStream_t);
template hipError_t launch_attn_probs<bf16>(const AttnArgs&, float*, int64_t, int64_t, hipStream_t);
