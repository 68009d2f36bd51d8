// Fused tail of a transformer layer (bf16 perf path):
//
//   x' = x + O . Wo^T                        attention output projection + residual (modules.py:96-110,
//                                              :262 / :272, proj has no bias)
//   x  = x' + W2 . GELU(W1 . LayerNorm(x'))  ffn_block + residual (modules.py:9-21, :274)
//
// One workgroup of 8 waves owns R = 16*MT rows (MT = 9: 144 rows, one workgroup per CU), so every
// weight byte streamed from L2 feeds 144 rows instead of the 64 of the separate row-panel / FFN
// kernels, and x' never goes to HBM (the unfused pair wrote x' and read it back: 2 x 33 MB per
// 32k rows, one launch more).
//
// Wave w owns output columns 32w .. 32w+31 of EVERY row of the workgroup.  Its accumulators start
// as the residual x, take the out-projection, then (after the LayerNorm) the three FFN-down
// slices: acc[i][j] is the 16x16 C^T tile (output columns 32w + 16i .., rows 16j ..), a lane
// holding 4 consecutive columns of one row (operands swapped: C^T = W . A^T).
//   LayerNorm(x'): row sums of acc over the wave's 32 columns, cross-wave through LDS (two passes:
//                  mean, then the centred variance), normalised rows -> bf16 panel P in LDS.
//   FFN in 3 hidden slices of 256: up (K 256 from P) -> GELU -> bf16 slice H in LDS -> down
//                  (K 256 of W2) accumulated into acc.  One barrier before H is overwritten, one
//                  after it is written; waves drift freely inside each k-loop.
// Weights come straight from L2 into registers in the packed row-panel layout (k_misc.hip
// pack_rowpanel: fragment (k-step, 16-row group) = 1 KiB contiguous), NPF k-steps ahead, as one
// stream over Wo (8 k-steps), then W1 slice s (8), W2 slice s (8) for s = 0..2.
// LDS (MT = 9): P 72 KiB + H 72 KiB (the O panel at the start, then the hidden slices) + 2 x 4.5 KiB
// row partials = 153 KiB.
#include <cstdlib>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

constexpr int D = 256;
constexpr int ROWB = D * 2;  // bf16 row of the panel / of a hidden slice: 512 B = 32 chunks
// weight prefetch depth NPF (k-steps, a template parameter): a 64-row k-step is only ~256 MFMA
// cycles per SIMD, so 2 in flight leave the L2 round trip exposed; 8 in flight cost 48 VGPRs,
// which drops the 64-row kernels from two workgroups per CU to one

// weight prefetch depth (k-steps in flight) of the production instantiations: the block kernels sit at
// 124 VGPRs (two workgroups per CU need <= 128), the LN-projection kernels at 90-100
#ifndef BLK_NPF
#define BLK_NPF 2
#endif
#ifndef LNP_NPF
#define LNP_NPF 2
#endif

template <int MT> struct Blk {
  static constexpr int R = 16 * MT;
  static constexpr int OFF_H = R * ROWB;
  static constexpr int OFF_RED = 2 * R * ROWB;  // [2][R][8] fp32 per-wave row partials
  static constexpr int OFF_GB = OFF_RED + 2 * R * 8 * 4;  // LayerNorm gamma / beta
  static constexpr int LDS = OFF_GB + 2 * D * 4;
};

// 16-B chunk c of row `row`: rows are 512 B (= 0 mod 256) apart, so XOR with row%16 spreads an
// MFMA fragment read (16 rows, lane groups of ds_read_b128) over distinct bank groups
VAP_DEV int xswz(int row, int c) { return c ^ (row & 15); }

// Row j*16 + l16 of a panel from the accumulator layout: a / b = the lane's 4 columns 32w + 4lg .. and
// 32w + 16 + 4lg .. as packed bf16.  v_permlane16_swap trades the two 16-column blocks between lane
// groups, so each lane holds 8 consecutive columns (32w + 16(lg & 1) + 8(lg >> 1) ..) and writes them as
// ONE 16-B chunk: conflict-free (8-lane groups of ds_write_b128 cover 8 distinct rows' swizzled chunks),
// where the two 8-B halves per lane put two lanes of each 16-lane group on one bank pair.
VAP_DEV void panel_put(unsigned char* img, int row, int w, int lg, u32x2 a, u32x2 b) {
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const auto sw = __builtin_amdgcn_permlane16_swap(a[d], b[d], false, false);
    a[d] = sw[0];
    b[d] = sw[1];
  }
  const int c = w * 4 + (lg & 1) * 2 + (lg >> 1);
  *(u32x4*)(img + row * ROWB + xswz(row, c) * 16) = u32x4{a[0], a[1], b[0], b[1]};
}

// GELU in sigmoid form, x * sigmoid(-x (c1 + c2 x^2) ln 2), with c1 / c2 fitted to the erf GELU
// (max |error| 2.7e-4 over the reals, below half a bf16 ulp for |x| >= 0.14): one v_exp + one v_rcp
// + 5 VALU.  Large negative x: exp2 -> +inf, rcp -> 0, result -0; large positive: x.
VAP_DEV float gelu_sig(float x) {
  const float u = x * __builtin_fmaf(x * x, -0.10012561f, -2.3087653f);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
}

// Byte offsets (from element `base`) of rows mf, mf + 16, .., mf + 16 (n - 1) of a row set whose
// row m sits at element (m / rps) * seq + (m % rps) * ld (rps = 0: m * ld), esz-byte elements: one
// division, then stepping.  Rows >= M get an offset outside every buffer resource (reads 0, stores
// drop).
VAP_DEV void rows16_off(int mf, int M, int rps, int64_t seq, int64_t ld, int64_t base, int esz, uint32_t* out, int n) {
  int sq = 0, t = mf;
  if (rps) {
    sq = mf / rps;
    t = mf - sq * rps;
  }
  for (int k = 0; k < n; ++k) {
    const int m = mf + 16 * k;
    const int64_t e = rps ? (int64_t)sq * seq + (int64_t)t * ld : (int64_t)m * ld;
    out[k] = m < M ? (uint32_t)((e - base) * esz) : 0x80000000u;
    t += 16;
    if (rps)
      while (t >= rps) {
        t -= rps;
        ++sq;
      }
  }
}

// LayerNorm of the R rows held in acc (wave w: columns 32w .. 32w+31; lane: row j*16 + l16, columns
// 32w + 16i + 4lg ..) -> bf16 panel P (XOR-swizzled rows), gamma / beta from GB[0..255] / GB[256..511].
// Row partials over the wave's 32 columns are summed over the 4 lane groups with permlane swaps
// (VALU, no LDS round trip), then exchanged as one LDS word per (row, wave): two passes (mean, then
// the centred variance), two barriers.  The caller's barrier publishes P.
template <int MT>
VAP_DEV void ln_panel(const f32x4 (&acc)[2][MT], float* red0, float* red1, const float* GB, unsigned char* P, int w,
                      int l16, int lg, float eps) {
  {  // every lane group writes the same partial
    auto gsum = [](float v) {  // sum over the 4 16-lane groups
      // inline asm: the builtins on two copies of one value were folded to a + a (ROCm 7.2 clang);
      // the s_nop covers the VALU-write -> permlane-read hazard the compiler cannot see
      float a = v, b = v;
      asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
      float c = a + b, d = c;
      asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(c), "+v"(d));
      return c + d;
    };
    auto rowtot = [&](const float* red, int j) {
      const f32x4 a = *(const f32x4*)(red + (j * 16 + l16) * 8), b = *(const f32x4*)(red + (j * 16 + l16) * 8 + 4);
      return ((a[0] + a[1]) + (a[2] + a[3])) + ((b[0] + b[1]) + (b[2] + b[3]));
    };
    float mean[MT], rstd[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) s += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
      red0[(j * 16 + l16) * 8 + w] = gsum(s);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      mean[j] = rowtot(red0, j) * (1.0f / D);
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = acc[i][j][e] - mean[j];
          s += d * d;
        }
      red1[(j * 16 + l16) * 8 + w] = gsum(s);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MT; ++j) rstd[j] = rsqrtf(rowtot(red1, j) * (1.0f / D) + eps);
    u32x2 yp[2][MT];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = w * 32 + i * 16 + lg * 4;
      const f32x4 ga = *(const f32x4*)(GB + n), be = *(const f32x4*)(GB + 256 + n);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const f32x4 y = (acc[i][j] - mean[j]) * rstd[j] * ga + be;
        yp[i][j] = pack_bf16x4(y[0], y[1], y[2], y[3]);
      }
    }
#pragma unroll
    for (int j = 0; j < MT; ++j) panel_put(P, j * 16 + l16, w, lg, yp[0][j], yp[1][j]);
  }
}

// diagnostics (VAP_BLOCK_STAMPS=1): wave 0 of workgroups 0, 32, .., 224 records s_memtime at [0] start,
// [1] O panel in LDS, [2] out-projection done, [3] LayerNorm panel complete, per slice s [4+4s] up done,
// [5+4s] GELU done + barrier, [6+4s] hidden slice written + barrier, [7+4s] down done, [16] stores
// issued, [17] stores complete
__device__ unsigned long long g_blk_stamps[8][24];

template <int MT, bool OPROJ, bool ST = false, int NPF = 2, int NP2 = 0, int NR2 = 0>
__global__ __launch_bounds__(512, 1) void block_kernel(BlockArgs g) {
  using C = Blk<MT>;
  constexpr int R = C::R;
  constexpr int Q0 = OPROJ ? 8 : 0;      // first FFN k-step of the weight stream
  constexpr int Q2 = Q0 + 48;            // first k-step of the fused next-layer projections
  constexpr int NQ = Q2 + 8 * (NP2 + NR2);  // Wo 8 + 3 x (W1 8 + W2 8) [+ Wp / Wr 8 per N tile]
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS];
#ifndef BLK_DIAG
#define BLK_DIAG 0
#endif
  // diagnostics (A/B builds only, outputs not meaningful): 1 no weight refills, 2 no GELU,
  // 4 A fragments read once per pass, 8 no O / x loads, 16 no stores
  unsigned char* P = smem;
  unsigned char* H = smem + C::OFF_H;
  float* red0 = (float*)(smem + C::OFF_RED);
  float* red1 = red0 + R * 8;
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * R;
  const int samp = (ST && (blockIdx.x & 31) == 0 && blockIdx.x < 256 && tid == 0) ? (int)(blockIdx.x >> 5) : -1;
  // phase boundary (+ a stamp in the diagnostics build): the scheduling barrier also keeps the
  // scheduler from mixing phases, which otherwise drives the 144-row variant into spills
  unsigned long long stv[18];  // wave-uniform: SGPRs
  auto stamp = [&](int k) {
    __builtin_amdgcn_sched_barrier(0);
    if (g.M < 0) asm volatile("s_nop 0");  // never taken: splits the block (basic-block boundary)
    if constexpr (ST) {
      stv[k] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp(0);

  auto roff = [&](int m, int64_t seq) -> int64_t {  // element offset of row m (256-wide rows)
    if (g.rows_per_seq == 0) return (int64_t)m * D;
    const int sq = m / g.rows_per_seq;
    return (int64_t)sq * seq + (int64_t)(m - sq * g.rows_per_seq) * D;
  };
  auto rows16 = [&](int mf, int64_t seq, int64_t base, int esz, uint32_t* out, int n) {
    rows16_off(mf, g.M, g.rows_per_seq, seq, D, base, esz, out, n);
  };

  // gamma / beta of the LayerNorm -> LDS (issued first: vmcnt counts in order)
  float* GB = (float*)(smem + C::OFF_GB);
  f32x4 gbv = {0.f, 0.f, 0.f, 0.f};
  if (tid < 128) gbv = *(const f32x4*)((tid < 64 ? g.gamma : g.beta) + (tid & 63) * 4);

  // ---------------------------------------------------------------- O panel (bf16) and residual rows
  // O first, so the out-projection waits for O only while x is still in flight; rows >= M read 0
  constexpr int OPT = R * 32 / 512;  // O chunks per thread (R multiple of 16)
  chunk16 ot[OPROJ ? OPT : 1];
  if constexpr (OPROJ) {
    const int64_t obase = roff(m0, g.o_seq);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(g.o + obase, 0x7FFFFFF0u);
    uint32_t oo[OPT];
    rows16(m0 + (tid >> 5), g.o_seq, obase, 2, oo, OPT);
#pragma unroll
    for (int k = 0; k < OPT; ++k) ot[k] = (BLK_DIAG & 8) ? chunk16{0u, 0u, 0u, 0u} : buf_load16(ro, oo[k] + (uint32_t)(tid & 31) * 16u, 0);
  }
  // lane's rows j*16 + l16 of x (recomputed for the stores at the end, not held live)
  const int64_t xbase = roff(m0, g.x_seq);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(g.x + xbase, 0x7FFFFFF0u);
  f32x4 acc[2][MT], xt[2][MT];
  {
    uint32_t xo[MT];
    rows16(m0 + l16, g.x_seq, xbase, 4, xo, MT);
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4 v = (BLK_DIAG & 8) ? f32x4{0.f, 0.f, 0.f, 0.f} : __builtin_bit_cast(f32x4, buf_load16(rx, xo[j] + (uint32_t)(w * 32 + i * 16 + lg * 4) * 4u, 0));
        if constexpr (OPROJ) {
          xt[i][j] = v;
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
          acc[i][j] = v;
        }
      }
  }

  // ---------------------------------------------------------------- weight stream
  // weights through buffer resources: the fragment offset is the lane's 16 bytes plus a scalar part,
  // no per-load 64-bit address arithmetic on the VALU (the flat form spent ~170 VALU per workgroup)
  const __amdgpu_buffer_rsrc_t rWo = make_rsrc(g.Wo, 0x7FFFFFF0u), rW1 = make_rsrc(g.W1, 0x7FFFFFF0u),
                               rW2 = make_rsrc(g.W2, 0x7FFFFFF0u);
  const uint32_t wlo = (uint32_t)lane * 16u;
  auto wload = [&](int q, chunk16* r) {  // q static after unrolling
    int kidx;
    const bool o = OPROJ && q < Q0;
    bool second = false;
    __amdgpu_buffer_rsrc_t rs;
    if (o) {
      kidx = q;
      rs = rWo;
    } else if (q < Q2) {
      const int t = q - Q0, s = t >> 4, u = t & 15;
      second = u >= 8;
      kidx = s * 8 + (u & 7);
      rs = second ? rW2 : rW1;
    } else {  // fused next-layer projection tiles (Wp then Wr, back to back)
      kidx = q - Q2;
      rs = make_rsrc(g.Wp, 0x7FFFFFF0u);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = buf_load16(rs, wlo, (uint32_t)((kidx * 16 + 2 * w + i) * 1024));
  };
  chunk16 wr[NPF][2];
#pragma unroll
  for (int p = 0; p < NPF; ++p) wload(p, wr[p]);

  // one k-step: acc[i][j] += W fragment i x A fragment j (A rows j*16 + l16 of an LDS image)
  // fragment j of k-step ks sits at byte (j*16 + l16) * 512 + ((ks*4 + lg) ^ l16) * 16 = abase(j) ^ ks*64
  // (ks*4 only touches chunk bits 2..4 and lg the low two, so the XOR splits)
  const uint32_t afo = (uint32_t)(l16 * ROWB + (lg ^ l16) * 16);
  chunk16 afk[MT];
  auto kstep = [&](const unsigned char* img, int ks, int q, f32x4 (&c)[2][MT]) {
    chunk16 af[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      if (!(BLK_DIAG & 4) || ks == 0) afk[j] = *(const chunk16*)(img + j * 16 * ROWB + (afo ^ (uint32_t)(ks * 64)));
      af[j] = afk[j];
    }
    chunk16* wf = wr[q % NPF];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) c[i][j] = mfma_chunk<bf16>(wf[i], af[j], c[i][j]);
    // unconditional refill (the tail reloads the last step): a conditional load makes the
    // compiler's vmcnt bookkeeping drain the whole prefetch
    if (!(BLK_DIAG & 1)) wload(q + NPF < NQ ? q + NPF : NQ - 1, wf);
    // keep k-steps apart: left alone, the scheduler hoists later k-steps' fragment reads over
    // earlier MFMAs and spills (the other wave on the SIMD covers the read latency instead)
    __builtin_amdgcn_sched_barrier(0);
  };

  if constexpr (OPROJ) {
#pragma unroll
    for (int k = 0; k < OPT; ++k) {
      const int id = tid + k * 512, row = id >> 5, c = id & 31;
      *(chunk16*)(H + row * ROWB + xswz(row, c) * 16) = ot[k];
    }
    if (tid < 128) *(f32x4*)(GB + tid * 4) = gbv;
    __syncthreads();
    stamp(1);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) kstep(H, ks, ks, acc);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc[i][j] += xt[i][j];
    stamp(2);
  } else {
    if (tid < 128) *(f32x4*)(GB + tid * 4) = gbv;
  }

  // ---------------------------------------------------------------- LayerNorm(x') -> P
  ln_panel<MT>(acc, red0, red1, GB, P, w, l16, lg, g.eps);
  __syncthreads();  // P complete
  stamp(3);

  // ---------------------------------------------------------------- FFN, 3 hidden slices of 256
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    f32x4 up[2][MT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) up[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) kstep(P, ks, Q0 + 16 * s + ks, up);
    stamp(4 + 4 * s);
    u32x2 hb[2][MT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j)
        hb[i][j] = (BLK_DIAG & 2) ? pack_bf16x4(up[i][j][0], up[i][j][1], up[i][j][2], up[i][j][3])
                                  : pack_bf16x4(gelu_sig(up[i][j][0]), gelu_sig(up[i][j][1]), gelu_sig(up[i][j][2]),
                               gelu_sig(up[i][j][3]));
    __syncthreads();  // every wave is done reading H (the O panel / the previous slice)
    stamp(5 + 4 * s);
#pragma unroll
    for (int j = 0; j < MT; ++j) panel_put(H, j * 16 + l16, w, lg, hb[0][j], hb[1][j]);
    __syncthreads();  // slice s of the hidden complete
    stamp(6 + 4 * s);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) kstep(H, ks, Q0 + 16 * s + 8 + ks, acc);
    stamp(7 + 4 * s);
  }

  // ---------------------------------------------------------------- x = acc (fp32, in place)
  int z;  // opaque zero: the offsets are recomputed here rather than kept live from the prologue
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  {
    uint32_t xo[MT];
    rows16(m0 + l16 + z, g.x_seq, xbase, 4, xo, MT);
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        if (!(BLK_DIAG & 16)) buf_store16_wt(rx, xo[j] + (uint32_t)(w * 32 + i * 16 + lg * 4) * 4u, __builtin_bit_cast(u32x4, acc[i][j]));
    if (g.xb) {  // bf16 copy (the combinator's input after the last layer): same rows, half the bytes
      const __amdgpu_buffer_rsrc_t rb = make_rsrc(g.xb + xbase, 0x7FFFFFF0u);
#pragma unroll
      for (int j = 0; j < MT; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          buf_store8(rb, ((xo[j] >> 1) | (xo[j] & 0x80000000u)) + (uint32_t)(w * 32 + i * 16 + lg * 4) * 2u,
                     pack_bf16x4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]));
    }
  }
  if constexpr (NP2 > 0) {
    // ---------------------------------------------------------------- next layer: LN2(x) -> Q/K/V, x -> cross K/V
    // (the rows are already in the accumulators: no re-read of x, one launch less; modules.py:252-272)
    // lane-derived offsets rebuilt from an opaque zero: reusing the prologue's keeps them live
    // through the FFN (+20 VGPRs, half the occupancy)
    int z2;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z2));
    const int tidb = tid + z2, l16b = l16 + z2, lgb = lg + z2;
    // this phase's arguments read here from the kernel-argument segment through an opaque pointer: held
    // from the prologue they spill SGPRs into a VGPR
    using KA = const __attribute__((address_space(4))) BlockArgs*;
    KA ka = (KA)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    f32x4 gb2 = {0.f, 0.f, 0.f, 0.f};
    if (tidb < 128) gb2 = *(const f32x4*)((tidb < 64 ? ka->gamma2 : ka->beta2) + (tidb & 63) * 4);
    __syncthreads();  // every wave is done with P (slice 2's up), H (slice 2's down) and GB (the first LN)
    if (tidb < 128) *(f32x4*)(GB + tidb * 4) = gb2;
    if constexpr (NR2 > 0) {  // raw rows (bf16) -> H
#pragma unroll
      for (int j = 0; j < MT; ++j)
        panel_put(H, j * 16 + l16b, w, lgb, pack_bf16x4(acc[0][j][0], acc[0][j][1], acc[0][j][2], acc[0][j][3]),
                  pack_bf16x4(acc[1][j][0], acc[1][j][1], acc[1][j][2], acc[1][j][3]));
    }
    __builtin_amdgcn_sched_barrier(0);
    ln_panel<MT>(acc, red0, red1, GB, P, w, l16b, lgb, g.eps);
    __syncthreads();  // P (and the raw panel) complete
    __builtin_amdgcn_sched_barrier(0);
    auto roffl = [&](int m, int64_t seq, int64_t ld) -> int64_t {
      if (g.rows_per_seq == 0) return (int64_t)m * ld;
      const int sq = m / g.rows_per_seq;
      return (int64_t)sq * seq + (int64_t)(m - sq * g.rows_per_seq) * ld;
    };
#pragma unroll
    for (int p = 0; p < NP2 + NR2; ++p) {
      const bool raw = p >= NP2;
      const int nt = raw ? p - NP2 : p;
      f32x4 c[2][MT];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) c[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) kstep(raw ? H : P, ks, Q2 + 8 * p + ks, c);
      bf16* out = raw ? ka->cr : ka->cp;
      const int wd = raw ? NR2 : NP2;  // output row width in 256-wide tiles
      const int64_t ld = (int64_t)wd * D, seq = g.x_seq * wd;
      const int64_t cbase = roffl(m0, seq, ld);
      const __amdgpu_buffer_rsrc_t rc = make_rsrc(out + cbase, 0x7FFFFFF0u);
      uint32_t co[MT];
      rows16_off(m0 + l16b, g.M, g.rows_per_seq, seq, ld, cbase, 2, co, MT);
      const uint32_t col = (uint32_t)(nt * 256 + w * 32 + (lgb & 1) * 16 + (lgb >> 1) * 8);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        u32x2 a = pack_bf16x4(c[0][j][0], c[0][j][1], c[0][j][2], c[0][j][3]);
        u32x2 b = pack_bf16x4(c[1][j][0], c[1][j][1], c[1][j][2], c[1][j][3]);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto sw = __builtin_amdgcn_permlane16_swap(a[d], b[d], false, false);
          a[d] = sw[0];
          b[d] = sw[1];
        }
        if (!(BLK_DIAG & 16)) buf_store16(rc, co[j] + col * 2u, u32x4{a[0], a[1], b[0], b[1]});
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (ST) {
    stamp(16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(17);
    if (samp >= 0)
      for (int k = 0; k < 18; ++k) g_blk_stamps[samp][k] = stv[k];
  }
}

template <int MT>
hipError_t launch_mt(const BlockArgs& g, hipStream_t st) {
  const dim3 grid((g.M + 16 * MT - 1) / (16 * MT));
  static const bool stamps = getenv("VAP_BLOCK_STAMPS") != nullptr;
  if (g.np) {  // fused next-layer projections (the 64-row variant only: launch_block forces MT 4)
    if constexpr (MT == 4) {
      if (g.nr) hipLaunchKernelGGL((block_kernel<MT, true, false, BLK_NPF, 3, 2>), grid, dim3(512), 0, st, g);
      else hipLaunchKernelGGL((block_kernel<MT, true, false, BLK_NPF, 3, 0>), grid, dim3(512), 0, st, g);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (stamps && g.o) hipLaunchKernelGGL((block_kernel<MT, true, true>), grid, dim3(512), 0, st, g);
  else if (g.o) hipLaunchKernelGGL((block_kernel<MT, true, false, BLK_NPF>), grid, dim3(512), 0, st, g);
  else hipLaunchKernelGGL((block_kernel<MT, false, false, BLK_NPF>), grid, dim3(512), 0, st, g);
  return hipGetLastError();
}

}  // namespace

// rows per workgroup: 64 (MT 4: 70 KiB LDS and 126 VGPRs, so two workgroups share a CU and one's
// HBM phases overlap the other's matrix work: 40 us per 32k rows) unless a small `cus` asks for 144 rows (MT 9:
// one workgroup per CU, weights streamed once per 144 rows: 47 us, its HBM load / store phases
// exposed); `cus` = 0 selects the default, a positive count lets MT 9 take inputs that 2 x cus
// 64-row workgroups would not cover in one round
hipError_t launch_block(const BlockArgs& g, int cus, hipStream_t st) {
  if (g.M <= 0 || g.rows_per_seq < 0 || !g.x || !g.W1 || !g.W2 || (g.o && !g.Wo)) return hipErrorInvalidValue;
  if (g.np && (g.np != 3 || (g.nr != 0 && g.nr != 2) || !g.o || !g.Wp || !g.cp || !g.gamma2 || !g.beta2 ||
               (g.nr && !g.cr)))
    return hipErrorInvalidValue;
  const int mt = g.np ? 4 : (cus > 0 && cus < 64 && (g.M + 63) / 64 > 2 * cus ? 9 : 4);
  const int bm = 16 * mt;
  // a panel's rows must lie within the 2 GiB a buffer offset reaches from its first row
  const int64_t span = g.rows_per_seq ? (bm / g.rows_per_seq + 2) * g.x_seq + (int64_t)bm * D : (int64_t)bm * D;
  if (span * 4 >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
  auto span2 = [&](int64_t seq, int64_t ld) {
    return (g.rows_per_seq ? (bm / g.rows_per_seq + 2) * seq + (int64_t)bm * ld : (int64_t)bm * ld) * 2;
  };
  if (g.np && span2(g.x_seq * 3, 3 * D) >= 0x7FFFFFF0LL)
    return hipErrorInvalidValue;
  if (mt == 4) return launch_mt<4>(g, st);
  if (mt == 9) return launch_mt<9>(g, st);
  return hipErrorInvalidValue;
}

// diagnostics: copy the block-kernel phase stamps (8 sampled workgroups x 24) to host memory
hipError_t read_block_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blk_stamps), sizeof(g_blk_stamps), 0, hipMemcpyDeviceToHost);
}

// ------------------------------------------------------------------------------------------------
// LayerNorm'd projections of a transformer layer in one launch (bf16 perf path), the same row-block
// structure as block_kernel (8 waves, wave w owns columns 32w .. 32w+31 of every 256-wide output
// tile, R = 16*MT rows, weights straight from L2):
//   OPROJ:  x' = x + O . Wo^T stored back to x (fp32) and kept in registers; C_p = LN(x') . Wp^T
//           -- the stereo layer's self-attention out-projection + LN_src + cross Q (modules.py:262-269)
//   !OPROJ: C_p = LN(x) . Wp^T (QKV) and, NR > 0, C_r = x . Wr^T from the raw rows (the cross K/V of
//           modules.py:265-272 take the UN-normalised pre-layer x): x is read from HBM once.
// NP / NR = 256-wide N tiles of C_p / C_r.  bf16 outputs leave as 16-B stores: v_permlane16_swap
// trades the two 16-column blocks between lane groups so a lane holds 8 consecutive columns.
namespace {

// diagnostics (VAP_LNPROJ_STAMPS=1): wave 0 of workgroups 0, 64, .., 448 records s_memtime at [0] start,
// [1] O panel in LDS, [2] out-projection done, [3] LN panel complete, [4 + p] pass p's MFMAs done,
// [10 + p] pass p's stores issued, [16] all stores complete
__device__ unsigned long long g_lnp_stamps[8][24];

template <int MT, bool OPROJ, int NP, int NR, bool ST = false, int NPF = 2>
__global__ __launch_bounds__(512, 1) void lnproj_kernel(LnProjArgs g) {
  static_assert(!(OPROJ && NR), "the raw panel shares H with the O panel");
  using C = Blk<MT>;
  constexpr int R = C::R;
  constexpr int Q0 = OPROJ ? 8 : 0;
  constexpr int NQ = Q0 + 8 * (NP + NR);
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS];
  unsigned char* P = smem;
  unsigned char* H = smem + C::OFF_H;
  float* red0 = (float*)(smem + C::OFF_RED);
  float* red1 = red0 + R * 8;
  float* GB = (float*)(smem + C::OFF_GB);
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * R;
  const int rps = g.rows_per_seq;
  const int samp = (ST && (blockIdx.x & 63) == 0 && blockIdx.x < 512 && tid == 0) ? (int)(blockIdx.x >> 6) : -1;
  unsigned long long stv[17] = {};  // wave-uniform: SGPRs
  auto stamp = [&](int k) {
    if constexpr (ST) {
      __builtin_amdgcn_sched_barrier(0);
      stv[k] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp(0);
  auto roff = [&](int m, int64_t seq, int64_t ld) -> int64_t {
    if (rps == 0) return (int64_t)m * ld;
    const int sq = m / rps;
    return (int64_t)sq * seq + (int64_t)(m - sq * rps) * ld;
  };

  f32x4 gbv = {0.f, 0.f, 0.f, 0.f};
  if (tid < 128) gbv = *(const f32x4*)((tid < 64 ? g.gamma : g.beta) + (tid & 63) * 4);

  constexpr int OPT = R * 32 / 512;
  chunk16 ot[OPROJ ? OPT : 1];
  if constexpr (OPROJ) {
    const int64_t obase = roff(m0, g.o_seq, D);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(g.o + obase, 0x7FFFFFF0u);
    uint32_t oo[OPT];
    rows16_off(m0 + (tid >> 5), g.M, rps, g.o_seq, D, obase, 2, oo, OPT);
#pragma unroll
    for (int k = 0; k < OPT; ++k) ot[k] = buf_load16(ro, oo[k] + (uint32_t)(tid & 31) * 16u, 0);
  }
  const int64_t xbase = roff(m0, g.x_seq, D);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(g.x + xbase, 0x7FFFFFF0u);
  uint32_t xo[MT];
  rows16_off(m0 + l16, g.M, rps, g.x_seq, D, xbase, 4, xo, MT);
  // accumulators start as x (OPROJ: the out-projection adds onto them; x is issued after O, so the
  // O panel can land while x is in flight)
  f32x4 acc[2][MT];
#pragma unroll
  for (int j = 0; j < MT; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      acc[i][j] = __builtin_bit_cast(f32x4, buf_load16(rx, xo[j] + (uint32_t)(w * 32 + i * 16 + lg * 4) * 4u, 0));

  // weights through buffer resources (see block_kernel)
  const __amdgpu_buffer_rsrc_t rWo = make_rsrc(g.Wo, 0x7FFFFFF0u), rWp = make_rsrc(g.Wp, 0x7FFFFFF0u),
                               rWr = make_rsrc(g.Wr, 0x7FFFFFF0u);
  const uint32_t wlo = (uint32_t)lane * 16u;
  auto wload = [&](int q, chunk16* r) {
    int kidx;
    const bool o = OPROJ && q < Q0;
    bool rr = false;
    if (o) {
      kidx = q;
    } else {
      const int p = (q - Q0) >> 3;
      rr = p >= NP;
      kidx = (p < NP ? p : p - NP) * 8 + ((q - Q0) & 7);
    }
    const __amdgpu_buffer_rsrc_t rs = o ? rWo : rr ? rWr : rWp;
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = buf_load16(rs, wlo, (uint32_t)((kidx * 16 + 2 * w + i) * 1024));
  };
  chunk16 wr[NPF][2];
#pragma unroll
  for (int p = 0; p < NPF; ++p) wload(p, wr[p]);
  const uint32_t afo = (uint32_t)(l16 * ROWB + (lg ^ l16) * 16);
  auto kstep = [&](const unsigned char* img, int ks, int q, f32x4 (&c)[2][MT]) {
    chunk16 af[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) af[j] = *(const chunk16*)(img + j * 16 * ROWB + (afo ^ (uint32_t)(ks * 64)));
    chunk16* wf = wr[q % NPF];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) c[i][j] = mfma_chunk<bf16>(wf[i], af[j], c[i][j]);
    wload(q + NPF < NQ ? q + NPF : NQ - 1, wf);
    __builtin_amdgcn_sched_barrier(0);
  };

  if (tid < 128) *(f32x4*)(GB + tid * 4) = gbv;
  if constexpr (OPROJ) {
#pragma unroll
    for (int k = 0; k < OPT; ++k) {
      const int id = tid + k * 512, row = id >> 5, c = id & 31;
      *(chunk16*)(H + row * ROWB + xswz(row, c) * 16) = ot[k];
    }
    __syncthreads();
    stamp(1);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) kstep(H, ks, ks, acc);
    stamp(2);
    // x' back to HBM now (it is the residual the cross attention adds to)
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        buf_store16_wt(rx, xo[j] + (uint32_t)(w * 32 + i * 16 + lg * 4) * 4u, __builtin_bit_cast(u32x4, acc[i][j]));
  }
  if constexpr (NR > 0) {  // raw rows (bf16) -> H
#pragma unroll
    for (int j = 0; j < MT; ++j)
      panel_put(H, j * 16 + l16, w, lg, pack_bf16x4(acc[0][j][0], acc[0][j][1], acc[0][j][2], acc[0][j][3]),
                pack_bf16x4(acc[1][j][0], acc[1][j][1], acc[1][j][2], acc[1][j][3]));
  }
  __builtin_amdgcn_sched_barrier(0);
  ln_panel<MT>(acc, red0, red1, GB, P, w, l16, lg, g.eps);
  __syncthreads();  // P (and the raw panel) complete
  __builtin_amdgcn_sched_barrier(0);
  stamp(3);

  // ---------------------------------------------------------------- projections, one N tile per pass
#pragma unroll
  for (int p = 0; p < NP + NR; ++p) {
    const bool raw = p >= NP;
    const int nt = raw ? p - NP : p;
    f32x4 c[2][MT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) c[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) kstep(raw ? H : P, ks, Q0 + 8 * p + ks, c);
    stamp(4 + p);
    bf16* out = raw ? g.cr : g.cp;
    const int64_t ld = raw ? g.ldr : g.ldp, seq = raw ? g.cr_seq : g.cp_seq;
    const int64_t cbase = roff(m0, seq, ld);
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(out + cbase, 0x7FFFFFF0u);
    uint32_t co[MT];
    rows16_off(m0 + l16, g.M, rps, seq, ld, cbase, 2, co, MT);
    const uint32_t col = (uint32_t)(nt * 256 + w * 32 + (lg & 1) * 16 + (lg >> 1) * 8);
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      u32x2 a = pack_bf16x4(c[0][j][0], c[0][j][1], c[0][j][2], c[0][j][3]);
      u32x2 b = pack_bf16x4(c[1][j][0], c[1][j][1], c[1][j][2], c[1][j][3]);
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const auto sw = __builtin_amdgcn_permlane16_swap(a[d], b[d], false, false);
        a[d] = sw[0];
        b[d] = sw[1];
      }
      buf_store16(rc, co[j] + col * 2u, u32x4{a[0], a[1], b[0], b[1]});
    }
    stamp(10 + p);
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (ST) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(16);
    if (samp >= 0)
      for (int k = 0; k < 17; ++k) g_lnp_stamps[samp][k] = stv[k];
  }
}

template <int MT>
hipError_t launch_lnproj_mt(const LnProjArgs& g, hipStream_t st) {
  const dim3 grid((g.M + 16 * MT - 1) / (16 * MT));
  static const bool stamps = getenv("VAP_LNPROJ_STAMPS") != nullptr;
  if (stamps) {
    if (g.o && g.np == 1 && g.nr == 0) hipLaunchKernelGGL((lnproj_kernel<MT, true, 1, 0, true>), grid, dim3(512), 0, st, g);
    else if (!g.o && g.np == 3 && g.nr == 2)
      hipLaunchKernelGGL((lnproj_kernel<MT, false, 3, 2, true>), grid, dim3(512), 0, st, g);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (g.o && g.np == 1 && g.nr == 0) hipLaunchKernelGGL((lnproj_kernel<MT, true, 1, 0, false, LNP_NPF>), grid, dim3(512), 0, st, g);
  else if (!g.o && g.np == 3 && g.nr == 0) hipLaunchKernelGGL((lnproj_kernel<MT, false, 3, 0, false, LNP_NPF>), grid, dim3(512), 0, st, g);
  else if (!g.o && g.np == 3 && g.nr == 2) hipLaunchKernelGGL((lnproj_kernel<MT, false, 3, 2, false, LNP_NPF>), grid, dim3(512), 0, st, g);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}


// ------------------------------------------------------------------------------------------
// Combinator + vap_head (+ va_classifier) of 64 frames in one launch (bf16 path; modules.py:434-449,
// model.py:257-261; the VAD logits from the same bf16 rows):
//   h      = GELU(LN(x1 . Wa^T)) + GELU(LN(x2 . Wb^T))      (one shared LayerNorm, no biases)
//   logits = h . Wh^T + bh
// x1 / x2 are the two speakers' rows of the bf16 copy of x the last layer's block kernel writes.
// Same row-block structure as block_kernel (8 waves, wave w owns output columns 32w .. +31 of all
// 64 rows, weights streamed from L2 in the packed row-panel layout, A panels in LDS): both panels
// are loaded at once, h stays in registers between the two halves and reaches LDS once, as the
// head's A panel.  Replaces two LN+GELU GEMM launches and the head GEMM (43 + 56 + 26 us per step).
// ------------------------------------------------------------------------------------------
template <int MT>
__global__ __launch_bounds__(512, 1) void heads_kernel(HeadsArgs g) {
  constexpr int R = 16 * MT;
  constexpr int NQ = 24, NPF = 2;  // Wa 8 + Wb 8 + Wh 8 k-steps
  constexpr int OFF_P = R * ROWB, OFF_RED = 2 * R * ROWB, OFF_GB = OFF_RED + 2 * R * 8 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[OFF_GB + 4 * D * 4];
  unsigned char* H = smem;          // x1 panel, then h
  unsigned char* P = smem + OFF_P;  // x2 panel
  float* red0 = (float*)(smem + OFF_RED);
  float* red1 = red0 + R * 8;
  float* GB = (float*)(smem + OFF_GB);  // gamma | beta | head bias | VAD head weight
  const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, lg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * R;

  // frame m -> clip m / T, t = m % T; x1 row = clip's sequence 2c, x2 row = 2c + 1 (+ x_seq)
  const int64_t xbase = (int64_t)(m0 / g.T) * 2 * g.x_seq + (int64_t)(m0 % g.T) * D;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(g.x + xbase, 0x7FFFFFF0u);
  constexpr int OPT = R * 32 / 512;  // 16-B chunks per thread and panel
  chunk16 a1[OPT], a2[OPT];
  {
    uint32_t oo[OPT];
    rows16_off(m0 + (tid >> 5), g.M, g.T, 2 * g.x_seq, D, xbase, 2, oo, OPT);
#pragma unroll
    for (int k = 0; k < OPT; ++k) {
      a1[k] = buf_load16(rx, oo[k] + (uint32_t)(tid & 31) * 16u, 0);
      a2[k] = buf_load16(rx, oo[k] == 0x80000000u ? oo[k] : oo[k] + (uint32_t)(g.x_seq * 2 + (tid & 31) * 16), 0);
    }
  }
  f32x4 gbv = {0.f, 0.f, 0.f, 0.f};
  if (tid < 256)
    gbv = *(const f32x4*)((tid < 64 ? g.gamma : tid < 128 ? g.beta : tid < 192 ? g.hbias : g.vw) + (tid & 63) * 4);

  const __amdgpu_buffer_rsrc_t rWa = make_rsrc(g.Wa, 0x7FFFFFF0u), rWb = make_rsrc(g.Wb, 0x7FFFFFF0u),
                               rWh = make_rsrc(g.Wh, 0x7FFFFFF0u);
  const uint32_t wlo = (uint32_t)lane * 16u;
  auto wload = [&](int q, chunk16* r) {  // q static after unrolling (weights through buffer resources)
    const __amdgpu_buffer_rsrc_t rs = q < 8 ? rWa : q < 16 ? rWb : rWh;
    const int kidx = q & 7;
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = buf_load16(rs, wlo, (uint32_t)((kidx * 16 + 2 * w + i) * 1024));
  };
  chunk16 wr[NPF][2];
#pragma unroll
  for (int p = 0; p < NPF; ++p) wload(p, wr[p]);
  const uint32_t afo = (uint32_t)(l16 * ROWB + (lg ^ l16) * 16);
  auto kstep = [&](const unsigned char* img, int ks, int q, f32x4 (&c)[2][MT]) {
    chunk16 af[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) af[j] = *(const chunk16*)(img + j * 16 * ROWB + (afo ^ (uint32_t)(ks * 64)));
    chunk16* wf = wr[q % NPF];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) c[i][j] = mfma_chunk<bf16>(wf[i], af[j], c[i][j]);
    wload(q + NPF < NQ ? q + NPF : NQ - 1, wf);  // unconditional (see block_kernel)
    __builtin_amdgcn_sched_barrier(0);
  };

#pragma unroll
  for (int k = 0; k < OPT; ++k) {
    const int id = tid + k * 512, row = id >> 5, c = id & 31;
    *(chunk16*)(H + row * ROWB + xswz(row, c) * 16) = a1[k];
    *(chunk16*)(P + row * ROWB + xswz(row, c) * 16) = a2[k];
  }
  if (tid < 256) *(f32x4*)(GB + tid * 4) = gbv;
  __syncthreads();
  {  // va_classifier (model.py:257-259) of both speakers: 4 threads per (row, speaker), 64 columns each,
     // from the fp32 rows of x (g.xf, as the reference) or else the bf16 panels
    const int r = tid >> 3, sp = (tid >> 2) & 1, part = tid & 3;
    const int m = m0 + r;
    float dsum = 0.f;
    if (g.xf) {
      if (m < g.M) {
        const float* xr = g.xf + (int64_t)(m / g.T) * 2 * g.x_seq + (int64_t)(m % g.T) * D + sp * g.x_seq + part * 64;
        f32x4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = *(const f32x4*)(xr + 4 * k);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const f32x4 wv = *(const f32x4*)(GB + 768 + part * 64 + 4 * k);
          dsum += (v[k][0] * wv[0] + v[k][1] * wv[1]) + (v[k][2] * wv[2] + v[k][3] * wv[3]);
        }
      }
    } else {
      const unsigned char* img = sp ? P : H;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = part * 8 + k;
        const bf16x8 v = *(const bf16x8*)(img + r * ROWB + xswz(r, c) * 16);
        const f32x4 w0 = *(const f32x4*)(GB + 768 + c * 8), w1 = *(const f32x4*)(GB + 768 + c * 8 + 4);
        dsum += (((float)v[0] * w0[0] + (float)v[1] * w0[1]) + ((float)v[2] * w0[2] + (float)v[3] * w0[3])) +
                (((float)v[4] * w1[0] + (float)v[5] * w1[1]) + ((float)v[6] * w1[2] + (float)v[7] * w1[3]));
      }
    }
    dsum += __shfl_xor(dsum, 1, 64);
    dsum += __shfl_xor(dsum, 2, 64);
    const int64_t om = g.out_T ? (int64_t)(m / g.T) * g.out_T + g.out_f0 + m % g.T : m;
    if (part == 0 && m < g.M) g.vad[om * 2 + sp] = dsum + g.vb[0];
  }
  __builtin_amdgcn_sched_barrier(0);  // phases apart (mixed by the scheduler they held 178 VGPRs)

  auto gsum = [](float v) {  // sum over the 4 16-lane groups (inline asm: see ln_panel)
    float a = v, b = v;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    float c = a + b, d = c;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(c), "+v"(d));
    return c + d;
  };
  auto rowtot = [&](const float* red, int j) {
    const f32x4 a = *(const f32x4*)(red + (j * 16 + l16) * 8), b = *(const f32x4*)(red + (j * 16 + l16) * 8 + 4);
    return ((a[0] + a[1]) + (a[2] + a[3])) + ((b[0] + b[1]) + (b[2] + b[3]));
  };
  // GELU(LayerNorm(c)) of the rows (shared combinator LN, biased variance), accumulated into h
  auto ln_gelu = [&](const f32x4 (&c)[2][MT], f32x4 (&h)[2][MT], bool first) {
    float mean[MT], rstd[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) sm += (c[i][j][0] + c[i][j][1]) + (c[i][j][2] + c[i][j][3]);
      red0[(j * 16 + l16) * 8 + w] = gsum(sm);
    }
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      mean[j] = rowtot(red0, j) * (1.0f / D);
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = c[i][j][e] - mean[j];
          sm += d * d;
        }
      red1[(j * 16 + l16) * 8 + w] = gsum(sm);
    }
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < MT; ++j) rstd[j] = rsqrtf(rowtot(red1, j) * (1.0f / D) + g.eps);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = w * 32 + i * 16 + lg * 4;
      const f32x4 ga = *(const f32x4*)(GB + n), be = *(const f32x4*)(GB + 256 + n);
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const f32x4 y = (c[i][j] - mean[j]) * rstd[j] * ga + be;
        const f32x4 gy = {gelu_sig(y[0]), gelu_sig(y[1]), gelu_sig(y[2]), gelu_sig(y[3])};
        h[i][j] = first ? gy : h[i][j] + gy;
      }
    }
  };

  f32x4 acc[2][MT], h[2][MT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) kstep(H, ks, ks, acc);  // x1 . Wa^T
  __builtin_amdgcn_sched_barrier(0);
  ln_gelu(acc, h, true);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) kstep(P, ks, 8 + ks, acc);  // x2 . Wb^T
  __builtin_amdgcn_sched_barrier(0);
  ln_gelu(acc, h, false);
  __builtin_amdgcn_sched_barrier(0);
  // h -> bf16 panel (H: every wave finished its x1 k-steps before the LayerNorms' barriers)
#pragma unroll
  for (int j = 0; j < MT; ++j)
    panel_put(H, j * 16 + l16, w, lg, pack_bf16x4(h[0][j][0], h[0][j][1], h[0][j][2], h[0][j][3]),
              pack_bf16x4(h[1][j][0], h[1][j][1], h[1][j][2], h[1][j][3]));
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const f32x4 hb = *(const f32x4*)(GB + 512 + w * 32 + i * 16 + lg * 4);
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = hb;
  }
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) kstep(H, ks, 16 + ks, acc);  // h . Wh^T + bh
  if (g.out_T) {  // a frame range of every clip: rows clip * out_T + out_f0 + t
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = m0 + j * 16 + l16;
      if (m < g.M) {
        float* lr = g.logits + ((int64_t)(m / g.T) * g.out_T + g.out_f0 + m % g.T) * D + w * 32 + lg * 4;
#pragma unroll
        for (int i = 0; i < 2; ++i) *(f32x4*)(lr + i * 16) = acc[i][j];
      }
    }
    return;
  }
  // logits rows m (contiguous [M][256] fp32)
  const __amdgpu_buffer_rsrc_t rl = make_rsrc(g.logits + (int64_t)m0 * D, 0x7FFFFFF0u);
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = m0 + j * 16 + l16;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      buf_store16(rl, m < g.M ? (uint32_t)(((j * 16 + l16) * D + w * 32 + i * 16 + lg * 4) * 4) : 0x80000000u,
                  __builtin_bit_cast(u32x4, acc[i][j]));
  }
}
}  // namespace

// supported: (o, np 1, nr 0) out-proj + LN + cross Q; (no o, np 3, nr 0) LN + QKV; (no o, np 3, nr 2)
// LN + QKV and raw cross K/V.  64-row workgroups (two per CU)
hipError_t launch_lnproj(const LnProjArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.rows_per_seq < 0 || !g.x || !g.Wp || !g.cp || (g.o && !g.Wo) || (g.nr && (!g.Wr || !g.cr)))
    return hipErrorInvalidValue;
  constexpr int bm = 64;
  // a workgroup's rows must lie within the 2 GiB a buffer offset reaches from its first row
  auto span = [&](int64_t seq, int64_t ld, int esz) {
    return (g.rows_per_seq ? (bm / g.rows_per_seq + 2) * seq + (int64_t)bm * ld : (int64_t)bm * ld) * esz;
  };
  if (span(g.x_seq, D, 4) >= 0x7FFFFFF0LL || span(g.cp_seq, g.ldp, 2) >= 0x7FFFFFF0LL ||
      (g.nr && span(g.cr_seq, g.ldr, 2) >= 0x7FFFFFF0LL) || (g.o && span(g.o_seq, D, 2) >= 0x7FFFFFF0LL))
    return hipErrorInvalidValue;
  return launch_lnproj_mt<4>(g, st);
}

hipError_t read_lnproj_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lnp_stamps), sizeof(g_lnp_stamps), 0, hipMemcpyDeviceToHost);
}

hipError_t launch_heads(const HeadsArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.T <= 0 || g.out_T < 0 || (g.out_T && g.out_f0 + g.T > g.out_T) || g.out_f0 < 0 || !g.x || !g.Wa || !g.Wb || !g.Wh || !g.logits || !g.vw || !g.vb || !g.vad || g.x_seq % 8)
    return hipErrorInvalidValue;
  // a workgroup's rows lie within the 2 GiB a buffer offset reaches from its first row
  if ((64 / g.T + 2) * 2 * g.x_seq * 2 + 64 * D * 2 >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
  hipLaunchKernelGGL((heads_kernel<4>), dim3((g.M + 63) / 64), dim3(512), 0, st, g);
  return hipGetLastError();
}
