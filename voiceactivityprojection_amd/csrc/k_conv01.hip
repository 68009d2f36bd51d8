// Fused CPC conv0 -> ChannelNorm -> ReLU -> conv1 -> ChannelNorm -> ReLU (bf16 perf mode).
//
// Reference: CPCEncoder conv0/batchNorm0 and conv1/batchNorm1 (vap/encoder_components.py:83-86,
// 99-100), ChannelNorm (:62-70, unbiased variance over the 256 channels).
//
// The conv0 activation (256 ch x 64000 positions per speaker per 20 s: 4.2 GB bf16 at batch 64) is
// never written to HBM.  conv1 (k=8, s=4, p=2) output t reads conv0 positions 4t-2+j, j = 0..7.
// Split j = r + 4h (phase r = 0..3, half h = 0..1): for a tile of outputs [t0, t0+256) and a phase
// r, the needed positions are G_r[i] = x0[4(t0+i) - 2 + r], i = 0..256, and output row i uses G_r[i]
// (h = 0) and G_r[i+1] (h = 1).  The kernel makes G_r in 32-channel SLICES inside the conv1 MFMA
// stream (see conv01m_kernel's header); every conv0 position is generated once per tile (plus one
// halo row per phase).
//
// conv0 itself runs on the MFMA: z^T[c][p] = sum_k A[c][k] S[k][p] with a K = 32 split-bf16 layout
//   k  0..9 : A = w_hi[c],  S = s_hi[p]      k 10..19: A = w_hi[c], S = s_lo[p]
//   k 20..29: A = w_lo[c],  S = s_hi[p]      k 30, 31: A = b_hi[c], b_lo[c],  S = 1
// (~16-bit mantissa products; the dropped w_lo*s_lo term is ~2^-16 relative), with the ChannelNorm
// folded in:  w = g*(W0 - mean_c W0), b = g*(b0 - mean_c b0)  so  x0 = relu(rstd_p * z + beta0).
// rstd_p comes from the exact centred quadratic form  var = (s^T G s + 2 h.s + beta)/255,
// G = Wc^T Wc (10x10), h = Wc^T bc, beta = bc.bc  (Wc, bc = centred conv0 weights / bias), so the
// statistics need no pass over the 256 channels.  Padding positions (p < 0 or p >= L0) are zero rows.
//
// Earlier generations (whole-phase G images v2, four-wave slices v9, 16x16x32 MFMAs v10) were
// retired in round 3; DESIGN.md section 3.1 keeps their measurements.
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

struct C0Stat {  // layout of the c0stat float array (host-computed at weight packing)
  static constexpr int G = 0;     // 10x10 centred Gram matrix
  static constexpr int H = 100;   // 10
  static constexpr int BETA = 110;
  static constexpr int N = 112;
};

// timing diagnostics (VAP_CONV01_STAMPS=1): s_memtime at the phase boundaries of sampled
// workgroups, read back with vap_test_read_stamps(); the production instantiation records nothing
__device__ unsigned long long g_conv01_stamps[8][24];

VAP_DEV int sphys(int row, int c) { return (c + 2 * (row >> 2)) & 3; }  // 64-B slice / SV rows
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
VAP_DEV uint32_t relu_bf16x2(float a, float b) {  // bf16(max(x, 0)) for two values: cvt_pk + pk_max_i16
  const bf16x2_t h = __builtin_convertvector((f32x2){a, b}, bf16x2_t);
  s16x2 v = __builtin_bit_cast(s16x2, h);
  v = __builtin_elementwise_max(v, (s16x2){0, 0});
  return __builtin_bit_cast(uint32_t, v);
}
constexpr int BM2 = 256, BN = 256, NPOS2 = 272, GROWS2 = BM2 + 1;  // 17 position tiles of 16 (>= 257)
constexpr int WSEG2 = 20 * BM2 + 32;                            // 5152 waveform floats per tile
constexpr int I_SVN = 4 * NPOS2;                                // 1088 split-sample rows
constexpr int I_GSLOT = NPOS2 * 64;                             // 17408

// ------------------------------------------------------------------------------------------
// conv01m_kernel: the conv0 image in (phase, 32-channel) SLICES on 256-row tiles, eight waves.
// conv1's K for phase r is taps r and r+4 over 256 channels.  Ordered as units u = (r = u>>3,
// g = u&7) of one 32-channel group with both taps (two 32-deep k-steps), a unit needs only the slice
// G_r[:, 32g..+32) (257 rows x 64 B).  ChannelNorm-0 statistics are per position and closed-form,
// so a slice is independent of the other channels and is made two units ahead, inside the MFMA
// stream, instead of regenerating a whole-phase image between k-loops.
//   * wave w owns output channels 32w .. 32w+31 for all 256 rows (8 row tiles of the 32x32x16
//     MFMA, 128 accumulators in AGPRs through inline-asm "+a" MFMAs, so two waves share a SIMD and
//     the partner's MFMAs fill the gaps one wave leaves);
//   * W1 fragments are unique per wave and go straight from L2 into a two-set register ring one
//     unit ahead (k-step-major layout: one fragment = 1 KiB contiguous);
//   * ChannelNorm-0 folded into the conv0 operand: the prologue stores rstd_p * [s_hi | s_lo | s_hi |
//     1 1] (split-bf16 after scaling) and the conv0 MFMA starts from beta0, so a slice is
//     relu(MFMA) -> bf16 (v_pk_max_i16 on the packed bit patterns) with no per-position loads;
//   * three slice slots (slice v in slot v%3): slice u+2 is made during unit u into the slot of
//     slice u-1, so ONE barrier at the start of unit u publishes slice u+1 and frees that slot;
//   * slice work split by (channel tile ct = w & 1, position tiles w/2 + 4x; waves 0 and 1 also
//     make tile 16, the rows 256.. only output row 255 reads); padding positions are zeroed with a
//     per-lane validity mask;
//   * G slots use the swizzle chunk' = (chunk + row/4) mod 4: conflict-free ds_read_b128 for 32
//     consecutive rows (either tap offset) and for the slice stores of 16 rows;
//   * epilogue rows are one lane each (row = lane % 32 of a row tile, 16 channels per lane, the
//     other 16 in lane ^ 32): ChannelNorm-1 by one exchange of per-wave (mean, M2) pairs, 16-B
//     stores via v_permlane32_swap.
// The waveform segment (prologue only) shares its LDS with slot 2 and the epilogue's reduction area.
// ------------------------------------------------------------------------------------------
constexpr int K_OFF_G = 0;                                    // 3 slots of 272 x 64 B
constexpr int K_OFF_RED = 3 * I_GSLOT;                        // 52224: [256 rows][8 waves] f32 (epilogue)
constexpr int K_OFF_WV = 2 * I_GSLOT;                         // 34816: over slot 2 + red (prologue)
constexpr int K_OFF_SV = K_OFF_RED + BM2 * 8 * 4;             // 60416
constexpr int K_OFF_C0 = K_OFF_SV + I_SVN * 64;               // 130048
constexpr int K_OFF_BE = K_OFF_C0 + 256 * 64;                 // 146432
constexpr int K_LDS = K_OFF_BE + 4 * 256 * 4;                 // 150528
static_assert(K_OFF_WV + WSEG2 * 4 <= K_OFF_SV, "conv01 waveform alias");
static_assert(K_LDS <= 163840, "conv01 LDS");

typedef float f32x16 __attribute__((ext_vector_type(16)));
VAP_DEV int gphys(int row, int c) { return (c + (row >> 2)) & 3; }
VAP_DEV int c1_lane() {  // the lane id by volatile asm: values derived from it are not hoisted
  int ln;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
  return ln;
}
VAP_DEV void mfma32_acc(f32x16& c, const chunk16& a, const chunk16& b) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <bool STAMPS>
__global__ __launch_bounds__(512, 1) void conv01m_kernel(const float* __restrict__ wav, int64_t N, int L0,
                                                        const chunk16* __restrict__ c0w, const float* __restrict__ c0stat,
                                                        const float* __restrict__ beta0, const bf16* __restrict__ W1,
                                                        const float* __restrict__ b1, const float* __restrict__ g1,
                                                        const float* __restrict__ be1, bf16* __restrict__ out,
                                                        int64_t out_seq_stride, int r0, int r1) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[K_LDS];
  unsigned char* G = smem + K_OFF_G;
  unsigned char* SV = smem + K_OFF_SV;
  unsigned char* C0 = smem + K_OFF_C0;
  float* BE = (float*)(smem + K_OFF_BE);
  float* EP = BE + 256;
  float* WV = (float*)(smem + K_OFF_WV);
  float* red = (float*)(smem + K_OFF_RED);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // output channels 32w..32w+31, all 256 rows
  const int ct = w & 1, pq = w >> 1;                        // slice work: channel tile, position tiles pq + 4x
  const bool p16 = w < 2;                                   // ... and tile 16 (rows 256.., read by row 255 only)
  const int s = blockIdx.y;
  const int t0 = r0 + blockIdx.x * BM2;
  const int samp = (STAMPS && (blockIdx.x == 0 || blockIdx.x == 3) && s < 4) ? (s * 2 + (blockIdx.x == 3)) : -1;
  unsigned long long stv[10], rt0 = 0;
  int nst = 0;
  if constexpr (STAMPS) rt0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz: the clock held = d(memtime) / d(rt)
  auto stamp = [&]() {
    if constexpr (STAMPS) {
      __builtin_amdgcn_sched_barrier(0);
      if (nst < 10) stv[nst] = __builtin_amdgcn_s_memtime();
      ++nst;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp();

  // W1 fragment (A of the 32x32x16): channel 32w + lane%32, k 16kh + 8(lane/32) of a 32-deep k-step
  const __amdgpu_buffer_rsrc_t wrs = make_rsrc(W1, 64 * 256 * 64);
  const uint32_t wlo = (uint32_t)((w * 32 + (lane & 31)) * 64 + (lane >> 5) * 16);
  auto wload = [&](int u, chunk16* wf) {  // unit u: [h * 2 + kh] = k-step (u, h), k half kh
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kk = ((u >> 3) + 4 * h) * 8 + (u & 7);
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) wf[h * 2 + kh] = buf_load16(wrs, wlo, (uint32_t)(kk * 16384 + kh * 32));
    }
  };

  // ---------------- prologue
  {
    const __amdgpu_buffer_rsrc_t wr = make_rsrc(wav + (int64_t)s * N, (uint32_t)(N * 4));
    const int xb = 20 * t0 - 13;  // first sample of the segment (negative offsets read as zero)
    uint32_t wv[11];
#pragma unroll
    for (int k = 0; k < 11; ++k)
      wv[k] = __builtin_amdgcn_raw_buffer_load_b32(wr, (int)((uint32_t)(xb + tid + 512 * k) * 4u), 0, 0);
    chunk16 c0[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) c0[i] = c0w[tid + i * 512];
    f32x4 ep = {0.f, 0.f, 0.f, 0.f};
    if (tid < 64) ep = ((const f32x4*)beta0)[tid];
    else if (tid < 128) ep = ((const f32x4*)b1)[tid - 64];
    else if (tid < 192) ep = ((const f32x4*)g1)[tid - 128];
    else if (tid < 256) ep = ((const f32x4*)be1)[tid - 192];
#pragma unroll
    for (int k = 0; k < 11; ++k)
      if (tid + 512 * k < WSEG2) WV[tid + 512 * k] = __builtin_bit_cast(float, wv[k]);
#pragma unroll
    for (int i = 0; i < 2; ++i) ((chunk16*)C0)[tid + i * 512] = c0[i];
    if (tid < 256) ((f32x4*)BE)[tid] = ep;
  }
  chunk16 W[2][4];  // W1 register ring: unit u in set u % 2, loaded one unit ahead
  wload(0, W[0]);
  __syncthreads();
  stamp();  // waveform segment in LDS

  for (int j = tid; j < I_SVN; j += 512) {
    const int r = j / NPOS2, i = j - r * NPOS2;
    const int p = 4 * (t0 + i) - 2 + r;
    const bool valid = i < GROWS2 && p >= 0 && p < L0;
    float sm[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) sm[k] = WV[min(20 * i + 5 * r + k, WSEG2 - 1)];
    float q = c0stat[C0Stat::BETA];
#pragma unroll
    for (int a = 0; a < 10; ++a) {
      float ga = fmaf(c0stat[C0Stat::G + a * 10 + a], sm[a], 2.0f * c0stat[C0Stat::H + a]);
#pragma unroll
      for (int b = a + 1; b < 10; ++b) ga = fmaf(2.0f * c0stat[C0Stat::G + a * 10 + b], sm[b], ga);
      q = fmaf(ga, sm[a], q);
    }
    const float rs = valid ? rsqrtf(fmaxf(q, 0.f) * (1.0f / 255.0f) + 1e-5f) : 0.f;
    bf16 hi[10], lo[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const float x = rs * sm[k];
      hi[k] = (bf16)x;
      lo[k] = (bf16)(x - (float)hi[k]);
    }
    const bf16 rb = (bf16)rs;
    const bf16x8 v[4] = {{hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]},
                         {hi[8], hi[9], lo[0], lo[1], lo[2], lo[3], lo[4], lo[5]},
                         {lo[6], lo[7], lo[8], lo[9], hi[0], hi[1], hi[2], hi[3]},
                         {hi[4], hi[5], hi[6], hi[7], hi[8], hi[9], rb, rb}};
    unsigned char* row = SV + j * 64;
#pragma unroll
    for (int c = 0; c < 4; ++c) *(bf16x8*)(row + sphys(j, c) * 16) = v[c];
  }

  // validity of this lane's position in slice tile x (pq + 4x, x < 4; 16 for x = 4) of phase r: bit 5r + x
  uint32_t vmask = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      const int pt = x == 4 ? 16 : pq + 4 * x;
      const int p = 4 * (t0 + pt * 16 + (lane & 15)) - 2 + r;
      vmask |= (uint32_t)(p >= 0 && p < L0) << (5 * r + x);
    }
  __syncthreads();
  stamp();  // split-sample rows built

  // ---- slice v (phase v>>3, channel group v&7) -> slot v%3; this wave makes channel tile ct
  auto read_c0 = [&](int v, chunk16& c0, f32x4& bt) {
    const int g = v & 7;
    c0 = ((const chunk16*)C0)[((2 * g + ct) * 16 + (lane & 15)) * 4 + (lane >> 4)];
    bt = *(const f32x4*)(BE + (2 * g + ct) * 16 + 4 * (lane >> 4));
  };
  auto read_sv = [&](int v, int x) -> chunk16 {
    const int pt = x == 4 ? 16 : pq + 4 * x;
    const int jj = ((v >> 3) & 3) * NPOS2 + pt * 16 + (lane & 15);
    return *(const chunk16*)(SV + jj * 64 + sphys(jj, lane >> 4) * 16);
  };
  auto pstore = [&](auto slc, int v, int x, const f32x4& z) {
    const int pt = x == 4 ? 16 : pq + 4 * x;
    const int prow = pt * 16 + (lane & 15);
    const uint32_t m = 0u - ((vmask >> (5 * ((v >> 3) & 3) + x)) & 1u);
    unsigned char* gs = G + decltype(slc)::value * I_GSLOT;
    const u32x2 o = {relu_bf16x2(z[0], z[1]) & m, relu_bf16x2(z[2], z[3]) & m};
    const int lc = 2 * ct + (lane >> 5);
    *(u32x2*)(gs + prow * 64 + gphys(prow, lc) * 16 + ((lane >> 4) & 1) * 8) = o;
  };
#pragma unroll
  for (int v = 0; v < 2; ++v) {  // slices 0 and 1
    chunk16 c0;
    f32x4 bt;
    read_c0(v, c0, bt);
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      if (x == 4 && !p16) break;
      const chunk16 sv = read_sv(v, x);
      if (v == 0) pstore(std::integral_constant<int, 0>{}, v, x, mfma_chunk<bf16>(c0, sv, bt));
      else pstore(std::integral_constant<int, 1>{}, v, x, mfma_chunk<bf16>(c0, sv, bt));
    }
  }

  // [row tile] of C^T (32 channels x 32 rows), in AGPRs; they start at the conv1 bias (lane element
  // e: channel 32w + 8(e/4) + 4(lane/32) + e%4), written here with the wait states the first MFMA
  // reading them as SrcC needs (the MFMAs are inline asm, invisible to the hazard recognizer)
  f32x16 acc[8];
  {
    f32x4 bb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bb[q] = *(const f32x4*)(EP + w * 32 + 4 * (lane >> 5) + 8 * q);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = bb[e >> 2][e & 3];
    asm volatile("s_nop 4" : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3]));
    asm volatile("s_nop 4" : "+a"(acc[4]), "+a"(acc[5]), "+a"(acc[6]), "+a"(acc[7]));
  }

  // fragment n = 16h + 8kh + i: tap offset h, k half kh (chunks 2kh + lane/32), row tile i
  auto gread = [&](auto slc, int n) -> chunk16 {
    const unsigned char* gs = G + decltype(slc)::value * I_GSLOT;
    const int row = (n & 7) * 32 + (lane & 31) + (n >> 4);
    return *(const chunk16*)(gs + row * 64 + gphys(row, 2 * ((n >> 3) & 1) + (lane >> 5)) * 16);
  };
  constexpr int GA = 3;  // G fragments in flight ahead of their MFMA (the ring, GA + 1, must divide 32)
  chunk16 gf[GA + 1];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // slices 0, 1 published; WV (slot 2) free
#pragma unroll
  for (int n = 0; n < GA; ++n) gf[n] = gread(std::integral_constant<int, 0>{}, n);
  stamp();

  // unit u (slot u % 3 = SL, a compile-time constant so every LDS offset is an immediate)
#ifndef C01_DIAG
#define C01_DIAG 0
#endif
  auto unit = [&](const int u, auto slc, chunk16* wf, chunk16* wn1, const bool last1, const bool nosl_) {
    constexpr int SL = decltype(slc)::value;
    const bool nosl = nosl_ || (C01_DIAG & 1);  // diag 1: no slice production
    // B_u: own slice u+1 stores retired; W1 of unit u (issued one unit ago) landed
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr ((C01_DIAG & 2) == 0) __builtin_amdgcn_s_barrier();  // diag 2: no unit barrier
    __builtin_amdgcn_sched_barrier(0);
    if (!last1 && (C01_DIAG & 8) == 0) wload(u + 1, wn1);  // diag 8: no W1 refill
    const int v = u + 2;
    chunk16 c0, sv;
    f32x4 bt, z;
    if (!nosl) read_c0(v, c0, bt);
#pragma unroll
    for (int n = 0; n < 32; ++n) {
      __builtin_amdgcn_sched_barrier(0);
      // slice v: tile x operands at MFMA 7x, conv0 MFMA at 7x+2, store at 7x+4 (tile 16: 28 / 30 / 31)
      if (!nosl && n % 7 == 0 && n / 7 < 4) sv = read_sv(v, n / 7);
      if (!nosl && n % 7 == 2 && n / 7 < 4) z = mfma_chunk<bf16>(c0, sv, bt);
      if (!nosl && n % 7 == 4 && n / 7 < 4) pstore(std::integral_constant<int, (SL + 2) % 3>{}, v, n / 7, z);
      if (!nosl && p16) {
        if (n == 28) sv = read_sv(v, 4);
        if (n == 30) z = mfma_chunk<bf16>(c0, sv, bt);
        if (n == 31) pstore(std::integral_constant<int, (SL + 2) % 3>{}, v, 4, z);
      }
      mfma32_acc(acc[n & 7], wf[n >> 3], gf[n % (GA + 1)]);
      if constexpr ((C01_DIAG & 4) == 0) {  // diag 4: G fragments re-used (no LDS reads)
        if (n + GA < 32) gf[(n + GA) % (GA + 1)] = gread(slc, n + GA);
        else if (!last1) gf[(n + GA) % (GA + 1)] = gread(std::integral_constant<int, (SL + 1) % 3>{}, n + GA - 32);
      }
    }
    if ((u & 7) == 7) stamp();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  for (int u = 0; u < 30; u += 6) {
    unit(u, I0{}, W[0], W[1], false, false);
    unit(u + 1, I1{}, W[1], W[0], false, false);
    unit(u + 2, I2{}, W[0], W[1], false, false);
    unit(u + 3, I0{}, W[1], W[0], false, false);
    unit(u + 4, I1{}, W[0], W[1], false, false);
    unit(u + 5, I2{}, W[1], W[0], false, false);
  }
  // units 30 and 31 have no slice to make (slices 32, 33 do not exist)
  unit(30, I0{}, W[0], W[1], false, true);
  unit(31, I1{}, W[1], W[0], true, true);

  // ---------------- epilogue: ChannelNorm (unbiased) over the 256 channels, ReLU, bf16
  // lane holds C[m = i*32 + lane%32][n = 32w + 8(e/4) + 4(lane/32) + e%4], e = 0..15 (+ b1).
  // One exchange of per-wave (mean, M2) pairs over the wave's 32 channels (Chan's parallel variance)
  // through the free G slots; gamma / beta read from LDS per row tile.
#pragma unroll
  for (int i = 0; i < 8; i += 4)  // MFMA -> VALU read of the accumulators
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3"
                 : "+a"(acc[i]), "+a"(acc[i + 1]), "+a"(acc[i + 2]), "+a"(acc[i + 3]));
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave done with the slots
  // lane-derived offsets are rebuilt per row tile from a volatile lane read: hoisted, they were
  // spilled in the prologue and every reload's vmcnt(0) waited for the previous row tile's stores
  float2* red2 = (float2*)G;                // [256 rows][8 waves] (mean, M2)
  auto val = [&](int i, int q) -> f32x4 {
    return f32x4{acc[i][4 * q], acc[i][4 * q + 1], acc[i][4 * q + 2], acc[i][4 * q + 3]};
  };
  auto xsum = [](float x) {  // x + x of lane ^ 32
    float a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
    return a + b;
  };
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    const f32x4 t = (val(i, 0) + val(i, 1)) + (val(i, 2) + val(i, 3));
    const float mw = xsum((t[0] + t[1]) + (t[2] + t[3])) * (1.0f / 32);
    // M2 of the wave's 32 channels as sum(x^2) - 32 mw^2: packed FMAs on the raw values (x - mw was
    // 16 scalar FMAs); in fp32 the cancellation is far below the bf16 output rounding
    f32x4 sq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) sq += val(i, q) * val(i, q);
    const float m2 = fmaxf(xsum((sq[0] + sq[1]) + (sq[2] + sq[3])) - 32.0f * mw * mw, 0.f);
    const int ln = c1_lane();
    if (ln < 32) red2[(i * 32 + ln) * 8 + w] = float2{mw, m2};
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  // 16-B stores: for channel blocks (2p, 2p+1) one v_permlane32_swap per dword gives lanes 0-31 the
  // 8 channels of block 2p and lanes 32-63 those of block 2p+1
  bf16* obase = out + (int64_t)s * out_seq_stride;
  const __amdgpu_buffer_rsrc_t orsc = make_rsrc(obase, (uint32_t)((int64_t)r1 * BN * 2));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    const int ln = c1_lane();
    const int cb = w * 32 + 4 * (ln >> 5);  // channel of e = 0; e -> cb + 8(e/4) + e%4
    const f32x4* rp = (const f32x4*)(red2 + (i * 32 + (ln & 31)) * 8);
    const f32x4 q0 = rp[0], q1 = rp[1], q2 = rp[2], q3 = rp[3];
    const float mean = (((q0[0] + q0[2]) + (q1[0] + q1[2])) + ((q2[0] + q2[2]) + (q3[0] + q3[2]))) * 0.125f;
    auto dev = [&](float mw) { return (mw - mean) * (mw - mean); };
    const float M2 = (((q0[1] + q0[3]) + (q1[1] + q1[3])) + ((q2[1] + q2[3]) + (q3[1] + q3[3]))) +
                     32.0f * (((dev(q0[0]) + dev(q0[2])) + (dev(q1[0]) + dev(q1[2]))) +
                              ((dev(q2[0]) + dev(q2[2])) + (dev(q3[0]) + dev(q3[2]))));
    float rstd = __builtin_amdgcn_rsqf(M2 * (1.0f / (BN - 1)) + 1e-5f);  // argument >= 1e-5: no denormal path
    float nmr = -mean * rstd;
    asm volatile("" : "+v"(rstd), "+v"(nmr));  // y = val * rstd + nmr: one packed FMA per 2 values
    const int t = t0 + i * 32 + (ln & 31);
    uint32_t pk[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 gg = *(const f32x4*)(EP + 256 + cb + 8 * q), ee = *(const f32x4*)(EP + 512 + cb + 8 * q);
      const f32x4 v = (val(i, q) * rstd + nmr) * gg + ee;
      pk[q][0] = relu_bf16x2(v[0], v[1]);
      pk[q][1] = relu_bf16x2(v[2], v[3]);
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const auto sw = __builtin_amdgcn_permlane32_swap(pk[2 * p][d], pk[2 * p + 1][d], false, false);
        pk[2 * p][d] = sw[0];
        pk[2 * p + 1][d] = sw[1];
      }
      const int col = w * 32 + 8 * (2 * p + (ln >> 5));
      const u32x4 o = {pk[2 * p][0], pk[2 * p][1], pk[2 * p + 1][0], pk[2 * p + 1][1]};
      buf_store16(orsc, t < r1 ? (uint32_t)(((int64_t)t * BN + col) * 2) : 0xFFFFFFF0u, o);
    }
  }
  if constexpr (STAMPS) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp();
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
    if (samp >= 0 && tid == 0) {
      for (int k = 0; k < 10 && k < nst; ++k) g_conv01_stamps[samp][k] = stv[k];
      g_conv01_stamps[samp][22] = rt0;
      g_conv01_stamps[samp][23] = rt1;
    }
  }
}

}  // namespace

hipError_t launch_conv01(const float* wav, int S, int64_t N, int L0, int L1, const bf16* c0w, const float* c0stat,
                         const float* beta0, const bf16* W1, const bf16* W1s, const float* b1, const float* g1,
                         const float* be1, bf16* out, int64_t out_seq_stride, hipStream_t st, int r0, int r1,
                         int grid_cap) {
  (void)W1;
  (void)grid_cap;
  if (r1 < 0) r1 = L1;
  if (S <= 0 || L1 <= 0 || r0 < 0 || r1 > L1 || r0 >= r1) return hipErrorInvalidValue;
  static const bool stamps = getenv("VAP_CONV01_STAMPS") != nullptr;
  const dim3 grid((r1 - r0 + BM2 - 1) / BM2, S);
  if (stamps)
    hipLaunchKernelGGL(conv01m_kernel<true>, grid, dim3(512), 0, st, wav, N, L0, (const chunk16*)c0w, c0stat, beta0, W1s,
                       b1, g1, be1, out, out_seq_stride, r0, r1);
  else
    hipLaunchKernelGGL(conv01m_kernel<false>, grid, dim3(512), 0, st, wav, N, L0, (const chunk16*)c0w, c0stat, beta0,
                       W1s, b1, g1, be1, out, out_seq_stride, r0, r1);
  return hipGetLastError();
}

// diagnostics: copy the conv01 v2 phase stamps (8 sampled workgroups x 24) to host memory
hipError_t read_conv01_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_conv01_stamps), sizeof(g_conv01_stamps), 0, hipMemcpyDeviceToHost);
}

// W [N][K] bf16 -> k-step-major [K/32][N][32]: each 32-deep k-step of all N rows is one contiguous
// block, so a conv01 W1 stage (256 rows x 64 B) is 16 KiB of consecutive lines spread over every L2
// channel (row-major rows 4 KiB apart hit the same channel)
__global__ void pack_kstep_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, int N, int K) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // output chunk of 8
  if (i >= (int64_t)N * K / 8) return;
  const int c = (int)(i & 3), n = (int)((i >> 2) % N), kk = (int)((i >> 2) / N);
  *(chunk16*)(out + i * 8) = *(const chunk16*)(in + (int64_t)n * K + kk * 32 + c * 8);
}
hipError_t launch_pack_kstep(const bf16* in, bf16* out, int N, int K, hipStream_t st) {
  if (K % 32 || N <= 0) return hipErrorInvalidValue;
  const int64_t chunks = (int64_t)N * K / 8;
  hipLaunchKernelGGL(pack_kstep_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, st, in, out, N, K);
  return hipGetLastError();
}
