// Fused CPC conv0 -> ChannelNorm -> ReLU -> conv1 -> ChannelNorm -> ReLU (bf16 perf mode).
//
// Reference: CPCEncoder conv0/batchNorm0 and conv1/batchNorm1 (vap/encoder_components.py:83-86,
// 99-100), ChannelNorm (:62-70, unbiased variance over the 256 channels).
//
// The conv0 activation (256 ch x 64000 positions per speaker per 20 s: 4.2 GB bf16 at batch 64) is
// never written to HBM.  conv1 (k=8, s=4, p=2) output t reads conv0 positions 4t-2+j, j = 0..7.
// Split j = r + 4h (phase r = 0..3, half h = 0..1): for a tile of 128 outputs [t0, t0+128) and a
// phase r, the needed positions are G_r[i] = x0[4(t0+i) - 2 + r], i = 0..128, and output row i uses
// G_r[i] (h = 0) and G_r[i+1] (h = 1).  Per phase the workgroup regenerates G_r (129 x 256 bf16) in
// LDS and runs the 512-deep K slice (taps r and r+4) of the conv1 GEMM against W1 tiles streamed
// from L2.  Every conv0 position is generated once per tile (plus one halo row per phase).
//
// conv0 itself runs on the MFMA: z^T[c][p] = sum_k A[c][k] S[k][p] with a K = 32 split-bf16 layout
//   k  0..9 : A = w_hi[c],  S = s_hi[p]      k 10..19: A = w_hi[c], S = s_lo[p]
//   k 20..29: A = w_lo[c],  S = s_hi[p]      k 30, 31: A = b_hi[c], b_lo[c],  S = 1
// (~16-bit mantissa products; the dropped w_lo*s_lo term is ~2^-16 relative), with the ChannelNorm
// folded in:  w = g*(W0 - mean_c W0), b = g*(b0 - mean_c b0)  so  x0 = relu(rstd_p * z + beta0).
// rstd_p comes from the exact centred quadratic form  var = (s^T G s + 2 h.s + beta)/255,
// G = Wc^T Wc (10x10), h = Wc^T bc, beta = bc.bc  (Wc, bc = centred conv0 weights / bias), so the
// statistics need no pass over the 256 channels.  Padding positions (p < 0 or p >= L0) are zero rows.
#include <cstdlib>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

constexpr int BM = 128, BN = 256, GROWS = BM + 1, GROWB = 512;  // G image: 129 rows x 256 ch bf16
constexpr int NPOS = 144;                                      // 9 position tiles of 16 (>= 129)
constexpr int SVROW = 80;                                      // padded split-sample row (32 bf16 + pad)
constexpr int BROWB = 128;                                     // W1 staging row: 64 k bf16
constexpr int OFF_G = 0;
constexpr int OFF_B = OFF_G + GROWS * GROWB;      // 66048
constexpr int OFF_SV = OFF_B + 2 * BN * BROWB;    // + 65536
constexpr int OFF_RS = OFF_SV + NPOS * SVROW;     // + 11520
constexpr int LDS_BYTES = OFF_RS + NPOS * 4;      // + 576 = 143680

VAP_DEV int gswz(int row, int c16) { return c16 ^ (row & 15); }      // 32 chunks per G row
// v2 G layout: chunk c of row r at position (c&1)*16 + ((c>>1) ^ r)&15 of the 512-B row -- chunks c and
// c+1 share a bank slot in opposite 256-B halves, so the slot depends on the row only and the
// fragment reads stay conflict-free for both tap offsets (rows m and m+1); the XOR of gswz is
// 2-way conflicted on the shifted rows.
VAP_DEV int gpos(int row, int c16) { return (c16 & 1) * 16 + (((c16 >> 1) ^ row) & 15); }
VAP_DEV int bswz(int row, int c) { return c ^ ((row >> 1) & 7); }    // 8 chunks per W1 staging row

struct C0Stat {  // layout of the c0stat float array (host-computed at weight packing)
  static constexpr int G = 0;     // 10x10 centred Gram matrix
  static constexpr int H = 100;   // 10
  static constexpr int BETA = 110;
  static constexpr int N = 112;
};

__global__ __launch_bounds__(512) void conv01_kernel(const float* __restrict__ wav, int64_t N, int L0, int L1,
                                                    const chunk16* __restrict__ c0w, const float* __restrict__ c0stat,
                                                    const float* __restrict__ beta0, const bf16* __restrict__ W1,
                                                    const float* __restrict__ b1, const float* __restrict__ g1,
                                                    const float* __restrict__ be1, bf16* __restrict__ out,
                                                    int64_t out_seq_stride, int r0, int r1) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  unsigned char* G = smem + OFF_G;
  unsigned char* Bt = smem + OFF_B;
  unsigned char* SV = smem + OFF_SV;
  float* RS = (float*)(smem + OFF_RS);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;
  const int s = blockIdx.y;
  const int t0 = r0 + blockIdx.x * BM;  // output rows [r0, r1) of conv1
  const float* src = wav + (int64_t)s * N;

  // conv0 A fragments of this wave: channel tiles 2w, 2w+1 (row c, k = 8(lane>>4)..+7)
  chunk16 a0f[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) a0f[j] = c0w[((2 * w + j) * 16 + (lane & 15)) * 4 + (lane >> 4)];
  float bet[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bet[j][e] = beta0[(2 * w + j) * 16 + 4 * (lane >> 4) + e];

  // W1 staging: 2048 chunks of 16 B per k-step (256 rows x 8), 4 per thread
  const bf16* bptr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + i * 512, row = id >> 3, c = id & 7;
    bptr[i] = W1 + (int64_t)row * 2048 + c * 8;
  }
  chunk16 rb[4];
  auto kbase = [](int q) {  // global k-step q (0..31): phase r = q>>3, half h = (q>>2)&1, sub (q&3)
    const int r = q >> 3, hh = (q >> 2) & 1, kk = q & 3;
    return (r + 4 * hh) * 256 + kk * 64;
  };
  auto gload = [&](int q) {
    const int kb = kbase(q);
#pragma unroll
    for (int i = 0; i < 4; ++i) rb[i] = *(const chunk16*)(bptr[i] + kb);
  };
  auto lstore = [&](int buf) {
    unsigned char* base = Bt + buf * BN * BROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * 512, row = id >> 3, c = id & 7;
      *(chunk16*)(base + row * BROWB + bswz(row, c) * 16) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  for (int r = 0; r < 4; ++r) {
    // ---------------- (a) split sample vectors + ChannelNorm statistics for the phase positions
    if (tid < NPOS) {
      const int i = tid;
      const int p = 4 * (t0 + i) - 2 + r;
      const bool valid = i < GROWS && p >= 0 && p < L0;
      float sm[10];
      const int64_t i0 = (int64_t)p * 5 - 3;
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        const int64_t ix = i0 + k;
        sm[k] = (valid && ix >= 0 && ix < N) ? src[ix] : 0.f;
      }
      bf16 hi[10], lo[10];
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        hi[k] = (bf16)sm[k];
        lo[k] = (bf16)(sm[k] - (float)hi[k]);
      }
      bf16x8 v0 = {hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]};
      bf16x8 v1 = {hi[8], hi[9], lo[0], lo[1], lo[2], lo[3], lo[4], lo[5]};
      bf16x8 v2 = {lo[6], lo[7], lo[8], lo[9], hi[0], hi[1], hi[2], hi[3]};
      bf16x8 v3 = {hi[4], hi[5], hi[6], hi[7], hi[8], hi[9], (bf16)1.0f, (bf16)1.0f};
      unsigned char* row = SV + i * SVROW;
      *(bf16x8*)(row + 0) = v0;
      *(bf16x8*)(row + 16) = v1;
      *(bf16x8*)(row + 32) = v2;
      *(bf16x8*)(row + 48) = v3;
      // var * 255 = s^T G s + 2 h.s + beta  (centred, exact in exact arithmetic)
      float q = c0stat[C0Stat::BETA];
#pragma unroll
      for (int a = 0; a < 10; ++a) {
        float ga = 2.0f * c0stat[C0Stat::H + a];
#pragma unroll
        for (int b = 0; b < 10; ++b) ga = fmaf(c0stat[C0Stat::G + a * 10 + b], sm[b], ga);
        q = fmaf(ga, sm[a], q);
      }
      RS[i] = valid ? rsqrtf(fmaxf(q, 0.f) * (1.0f / 255.0f) + 1e-5f) : -1.0f;
    }
    __syncthreads();  // (also: every wave finished reading the previous phase's G)

    // ---------------- (b) conv0 on the MFMA -> ChannelNorm/ReLU -> bf16 G image
#pragma unroll
    for (int pt = 0; pt < NPOS / 16; ++pt) {
      const int prow = pt * 16 + (lane & 15);  // position row of this lane's column
      const chunk16 bfr = *(const chunk16*)(SV + prow * SVROW + (lane >> 4) * 16);
      const float rs = RS[prow];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
        z = mfma_chunk<bf16>(a0f[j], bfr, z);
        if (prow < GROWS) {
          const int c = (2 * w + j) * 16 + 4 * (lane >> 4);  // 4 consecutive channels
          bf16x4 o4;
#pragma unroll
          for (int e = 0; e < 4; ++e) o4[e] = (bf16)(rs < 0.f ? 0.f : fmaxf(fmaf(rs, z[e], bet[j][e]), 0.f));
          *(bf16x4*)(G + prow * GROWB + gswz(prow, c >> 3) * 16 + (c & 7) * 2) = o4;
        }
      }
    }
    // stage the first W1 tile of this phase
    lstore(0);
    __syncthreads();

    // ---------------- (c) 8 k-steps of 64 over taps r (h = 0) and r + 4 (h = 1)
    for (int kq = 0; kq < 8; ++kq) {
      const int q = r * 8 + kq;
      const int cur = kq & 1;
      if (q + 1 < 32) gload(q + 1);
      const int hh = kq >> 2, kk = kq & 3;
      const unsigned char* bbase = Bt + cur * BN * BROWB;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        chunk16 af[4], bfr[4];
        const int c16 = kk * 8 + sub * 4 + (lane >> 4);  // chunk within the 512-B G row
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * 64 + i * 16 + (lane & 15) + hh;
          af[i] = *(const chunk16*)(G + row * GROWB + gswz(row, c16) * 16);
        }
        const int cb = sub * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = wn * 64 + j * 16 + (lane & 15);
          bfr[j] = *(const chunk16*)(bbase + row * BROWB + bswz(row, cb) * 16);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma_chunk<bf16>(af[i], bfr[j], acc[i][j]);
      }
      if (kq + 1 < 8) lstore(cur ^ 1);
      __syncthreads();
    }
  }

  // ---------------- epilogue: + b1, ChannelNorm (unbiased) over the 256 channels, ReLU, bf16
  const int colb = wn * 64 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float b = b1[colb + j * 16];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][j] += b;
  }
  float* red = (float*)Bt;  // [BM][4]
  float mean[4][4], rstd[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float sum = acc[i][0][e] + acc[i][1][e] + acc[i][2][e] + acc[i][3][e];
      sum += __shfl_xor(sum, 1, 64);
      sum += __shfl_xor(sum, 2, 64);
      sum += __shfl_xor(sum, 4, 64);
      sum += __shfl_xor(sum, 8, 64);
      if ((lane & 15) == 0) red[(wm * 64 + i * 16 + (lane >> 4) * 4 + e) * 4 + wn] = sum;
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f32x4 pr = *(const f32x4*)(red + (wm * 64 + i * 16 + (lane >> 4) * 4 + e) * 4);
      mean[i][e] = (pr[0] + pr[1] + pr[2] + pr[3]) * (1.0f / BN);
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = acc[i][j][e] - mean[i][e];
        ss += d * d;
      }
      ss += __shfl_xor(ss, 1, 64);
      ss += __shfl_xor(ss, 2, 64);
      ss += __shfl_xor(ss, 4, 64);
      ss += __shfl_xor(ss, 8, 64);
      if ((lane & 15) == 0) red[(wm * 64 + i * 16 + (lane >> 4) * 4 + e) * 4 + wn] = ss;
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f32x4 pr = *(const f32x4*)(red + (wm * 64 + i * 16 + (lane >> 4) * 4 + e) * 4);
      rstd[i][e] = rsqrtf((pr[0] + pr[1] + pr[2] + pr[3]) * (1.0f / (BN - 1)) + 1e-5f);
    }
  bf16* obase = out + (int64_t)s * out_seq_stride;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int t = t0 + wm * 64 + i * 16 + (lane >> 4) * 4 + e;
      if (t >= r1) continue;
      bf16* orow = obase + (int64_t)t * BN;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = colb + j * 16;
        const float v = (acc[i][j][e] - mean[i][e]) * rstd[i][e] * g1[col] + be1[col];
        orow[col] = (bf16)fmaxf(v, 0.f);
      }
    }
}

// ------------------------------------------------------------------------------------------
// v2 (default): the same fused math, restaged for the MI355X memory pipeline:
//   * W1 k-tiles (256 rows x 64 k) arrive by LDS-DMA (global_load_lds_dwordx4, swizzle applied to
//     the source address), two stages, raw s_barrier + vmcnt: the next tile's DMA stays in flight
//     across the MFMAs, the phase barriers and the conv0 regeneration;
//   * the tile's whole waveform segment (~10 KiB, every phase's samples) is loaded into LDS once, so
//     a phase's split samples / ChannelNorm statistics come from LDS instead of dependent global loads;
//   * operands swapped (C^T = W1 G^T): a lane owns 4 consecutive output channels of one row ->
//     8-byte bf16 stores (16 per lane instead of 64 two-byte stores), ChannelNorm row statistics by a
//     16-lane-stride shuffle + LDS.
// ------------------------------------------------------------------------------------------
constexpr int WSEG = 2592;                           // waveform floats per tile: 20*128 + 15 + 10 (+pad)
constexpr int B_OFF_G = 0;
constexpr int B_OFF_W = B_OFF_G + GROWS * GROWB;     // 66048: 2 W1 stages of 256 x 128 B
constexpr int B_OFF_SV = B_OFF_W + 2 * BN * BROWB;   // + 65536
constexpr int B_OFF_RS = B_OFF_SV + NPOS * SVROW;    // + 11520
constexpr int B_OFF_WV = B_OFF_RS + NPOS * 4;        // + 576
constexpr int B_LDS = B_OFF_WV + WSEG * 4;           // + 10368 = 154048
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr int WST = BN * 64;                          // v2 W1 stage: 256 rows x 64 B (4 stages = B_OFF_W area)
VAP_DEV int wswz(int row, int c) { return c ^ ((row >> 2) & 2); }  // 64-B rows: conflict-free b128 reads

VAP_DEV void lds_barrier() {  // LDS writes retired + workgroup barrier, without draining the DMA
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// timing diagnostics (VAP_CONV01_STAMPS=1): s_memtime at the phase boundaries of sampled
// workgroups, read back with vap_test_read_stamps(); the production instantiation records nothing
__device__ unsigned long long g_conv01_stamps[8][24];

template <bool STAMPS>
__global__ __launch_bounds__(512, 1) void conv01b_kernel(const float* __restrict__ wav, int64_t N, int L0,
                                                        const chunk16* __restrict__ c0w, const float* __restrict__ c0stat,
                                                        const float* __restrict__ beta0, const bf16* __restrict__ W1,
                                                        const float* __restrict__ b1, const float* __restrict__ g1,
                                                        const float* __restrict__ be1, bf16* __restrict__ out,
                                                        int64_t out_seq_stride, int r0, int r1) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[B_LDS];
  unsigned char* G = smem + B_OFF_G;
  unsigned char* Wt = smem + B_OFF_W;
  unsigned char* SV = smem + B_OFF_SV;
  float* RS = (float*)(smem + B_OFF_RS);
  float* WV = (float*)(smem + B_OFF_WV);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;  // 64 rows (t) x 64 output channels per wave
  const int s = blockIdx.y;
  const int t0 = r0 + blockIdx.x * BM;
  const float* src = wav + (int64_t)s * N;
  const unsigned char* W1b = (const unsigned char*)W1;
  // conv0 operand fragments of this wave (channel tiles 2w, 2w+1) and folded ChannelNorm shifts
  chunk16 a0f[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) a0f[j] = c0w[((2 * w + j) * 16 + (lane & 15)) * 4 + (lane >> 4)];
  float bet[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bet[j][e] = beta0[(2 * w + j) * 16 + 4 * (lane >> 4) + e];
  // sampled workgroups: block x in {0, 7}, sequence in {0, 1, 2, 3}
  const int samp = (STAMPS && (blockIdx.x == 0 || blockIdx.x == 7) && s < 4) ? (s * 2 + (blockIdx.x == 7)) : -1;
  unsigned long long stv[24];
  int nst = 0;
  auto stamp = [&]() {
    if constexpr (STAMPS) {
      __builtin_amdgcn_sched_barrier(0);
      if (nst < 24) stv[nst] = __builtin_amdgcn_s_memtime();
      ++nst;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp();

  // W1 DMA, 4 stages of 256 rows x 64 B (k 32 deep): a piece = 16 rows x 64 B; wave w fills pieces
  // 2w, 2w+1 of a 16-piece stage; lane -> (row 16p + lane/4, physical chunk lane%4) holding logical
  // chunk (lane%4) ^ wswz(row).  Three stages stay in flight (counted vmcnt).
  uint32_t woff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (w * 2 + i) * 16 + (lane >> 2);
    woff[i] = (uint32_t)(row * 2048 + wswz(row, lane & 3) * 8) * 2;
  }
  auto kbase = [](int q) {  // k-step q (0..63): phase q>>4, tap half (q>>3)&1, 32-channel group q&7
    return ((q >> 4) + 4 * ((q >> 3) & 1)) * 256 + (q & 7) * 32;
  };
  auto dma = [&](int q) {
    unsigned char* base = Wt + (q & 3) * WST;
    const uint32_t kb = (uint32_t)kbase(q) * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(W1b + (woff[i] + kb)), (lds_void_t*)(base + (w * 2 + i) * 1024), 16, 0, 0);
  };


  // the tile's waveform segment: samples 20*t0 - 13 + [0, WSEG) (zeros outside the signal)
  const int64_t xb = (int64_t)20 * t0 - 13;
  for (int i = tid; i < WSEG; i += 512) {
    const int64_t ix = xb + i;
    WV[i] = (ix >= 0 && ix < N) ? src[ix] : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // only the DMA ring uses vmcnt from here on
  dma(0);
  dma(1);
  dma(2);
  lds_barrier();
  stamp();

  f32x4 acc[4][4];  // [n tile][m tile] of C^T
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int r = 0; r < 4; ++r) {
    // ---------------- (a) split samples + ChannelNorm statistics of the phase positions (LDS only)
    if (tid < NPOS) {
      const int i = tid;
      const int p = 4 * (t0 + i) - 2 + r;
      const bool valid = i < GROWS && p >= 0 && p < L0;
      float sm[10];
#pragma unroll
      for (int k = 0; k < 10; ++k) sm[k] = WV[min(20 * i + 5 * r + k, WSEG - 1)];
      bf16 hi[10], lo[10];
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        hi[k] = (bf16)sm[k];
        lo[k] = (bf16)(sm[k] - (float)hi[k]);
      }
      bf16x8 v0 = {hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]};
      bf16x8 v1 = {hi[8], hi[9], lo[0], lo[1], lo[2], lo[3], lo[4], lo[5]};
      bf16x8 v2 = {lo[6], lo[7], lo[8], lo[9], hi[0], hi[1], hi[2], hi[3]};
      bf16x8 v3 = {hi[4], hi[5], hi[6], hi[7], hi[8], hi[9], (bf16)1.0f, (bf16)1.0f};
      unsigned char* row = SV + i * SVROW;
      *(bf16x8*)(row + 0) = v0;
      *(bf16x8*)(row + 16) = v1;
      *(bf16x8*)(row + 32) = v2;
      *(bf16x8*)(row + 48) = v3;
      float q = c0stat[C0Stat::BETA];
#pragma unroll
      for (int a = 0; a < 10; ++a) {
        float ga = 2.0f * c0stat[C0Stat::H + a];
#pragma unroll
        for (int b = 0; b < 10; ++b) ga = fmaf(c0stat[C0Stat::G + a * 10 + b], sm[b], ga);
        q = fmaf(ga, sm[a], q);
      }
      RS[i] = valid ? rsqrtf(fmaxf(q, 0.f) * (1.0f / 255.0f) + 1e-5f) : -1.0f;
    }
    lds_barrier();  // SV/RS ready; every wave done reading the previous phase's G
    stamp();

    // ---------------- (b) conv0 on the MFMA -> ChannelNorm/ReLU -> bf16 G image
#pragma unroll
    for (int pt = 0; pt < NPOS / 16; ++pt) {
      const int prow = pt * 16 + (lane & 15);
      const chunk16 bfr = *(const chunk16*)(SV + prow * SVROW + (lane >> 4) * 16);
      const float rs = RS[prow];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
        z = mfma_chunk<bf16>(a0f[j], bfr, z);
        if (prow < GROWS) {
          const int c = (2 * w + j) * 16 + 4 * (lane >> 4);
          bf16x4 o4;
#pragma unroll
          for (int e = 0; e < 4; ++e) o4[e] = (bf16)(rs < 0.f ? 0.f : fmaxf(fmaf(rs, z[e], bet[j][e]), 0.f));
          *(bf16x4*)(G + prow * GROWB + gpos(prow, c >> 3) * 16 + (c & 7) * 2) = o4;
        }
      }
    }
    lds_barrier();  // G ready
    stamp();

    // ---------------- (c) 16 k-steps of 32 over taps r (h = 0) and r + 4 (h = 1)
    for (int kq = 0; kq < 16; ++kq) {
      const int q = r * 16 + kq;
      __builtin_amdgcn_sched_barrier(0);
      // this wave's DMA of stage q landed: newer are stages q+1, q+2 (2 DMAs each, if issued)
      if (q + 2 < 64) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (q + 1 < 64) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's stage q landed; stage q-1's buffer fully read
      __builtin_amdgcn_sched_barrier(0);
      if (q + 3 < 64) dma(q + 3);   // into stage q-1's buffer
      const int hh = kq >> 3, kc = kq & 7;
      const unsigned char* wb = Wt + (q & 3) * WST;
      chunk16 gf[4], wf[4];
      const int c16 = kc * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + (lane & 15) + hh;
        gf[i] = *(const chunk16*)(G + row * GROWB + gpos(row, c16) * 16);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + j * 16 + (lane & 15);
        wf[j] = *(const chunk16*)(wb + row * 64 + wswz(row, lane >> 4) * 16);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = mfma_chunk<bf16>(wf[j], gf[i], acc[j][i]);
    }
    stamp();
  }

  // ---------------- epilogue: + b1, ChannelNorm (unbiased) over the 256 channels, ReLU, bf16
  // lane holds C[m = wm*64 + i*16 + lane%16][n = wn*64 + j*16 + (lane/16)*4 + e]
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // no DMA in flight; every wave done with the W1 stages (reused below)
  const int nb = wn * 64 + (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x4 b = *(const f32x4*)(b1 + nb + j * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] += b;
  }
  float* red = (float*)Wt;  // [BM][4 waves along N]
  float mean[4], rstd[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) sum += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    if ((lane >> 4) == 0) red[(wm * 64 + i * 16 + (lane & 15)) * 4 + wn] = sum;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 pr = *(const f32x4*)(red + (wm * 64 + i * 16 + (lane & 15)) * 4);
    mean[i] = (pr[0] + pr[1] + pr[2] + pr[3]) * (1.0f / BN);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = acc[j][i][e] - mean[i];
        ss += d * d;
      }
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if ((lane >> 4) == 0) red[(wm * 64 + i * 16 + (lane & 15)) * 4 + wn] = ss;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 pr = *(const f32x4*)(red + (wm * 64 + i * 16 + (lane & 15)) * 4);
    rstd[i] = rsqrtf((pr[0] + pr[1] + pr[2] + pr[3]) * (1.0f / (BN - 1)) + 1e-5f);
  }
  bf16* obase = out + (int64_t)s * out_seq_stride;
  // rows outer, column tiles inner: a wave completes each 128-B line of a row in consecutive stores
  // (column-outer order wrote ~1.9x the output bytes to HBM: partial lines left L2 between stores)
  f32x4 ga[4], be[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ga[j] = *(const f32x4*)(g1 + nb + j * 16);
    be[j] = *(const f32x4*)(be1 + nb + j * 16);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = t0 + wm * 64 + i * 16 + (lane & 15);
    if (t >= r1) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 v = (acc[j][i] - mean[i]) * rstd[i] * ga[j] + be[j];
      store4(obase + (int64_t)t * BN + nb + j * 16, fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f),
             fmaxf(v[3], 0.f));
    }
  }
  if constexpr (STAMPS) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp();
    if (samp >= 0 && tid == 0)
      for (int k = 0; k < 24 && k < nst; ++k) g_conv01_stamps[samp][k] = stv[k];
  }
}

// ------------------------------------------------------------------------------------------
// v3 (default): v2's staging with 4 waves (one per SIMD) of 64 rows x 128 channels each: per
// 32-deep step a wave reads 4 G + 8 W1 fragments for 32 MFMAs (v2: 4 + 4 for 16), halving the LDS
// read traffic per MFMA -- the G reads are inherently 2-way bank conflicted (the tap-shifted row
// offset), so LDS, not the MFMA pipe, bounded v2.
// v2: the same fused math, restaged for the MI355X memory pipeline:
//   * W1 k-tiles (256 rows x 64 k) arrive by LDS-DMA (global_load_lds_dwordx4, swizzle applied to
//     the source address), two stages, raw s_barrier + vmcnt: the next tile's DMA stays in flight
//     across the MFMAs, the phase barriers and the conv0 regeneration;
//   * the tile's whole waveform segment (~10 KiB, every phase's samples) is loaded into LDS once, so
//     a phase's split samples / ChannelNorm statistics come from LDS instead of dependent global loads;
//   * operands swapped (C^T = W1 G^T): a lane owns 4 consecutive output channels of one row ->
//     8-byte bf16 stores (16 per lane instead of 64 two-byte stores), ChannelNorm row statistics by a
//     16-lane-stride shuffle + LDS.
// ------------------------------------------------------------------------------------------



__global__ __launch_bounds__(256, 1) void conv01c_kernel(const float* __restrict__ wav, int64_t N, int L0,
                                                        const chunk16* __restrict__ c0w, const float* __restrict__ c0stat,
                                                        const float* __restrict__ beta0, const bf16* __restrict__ W1,
                                                        const float* __restrict__ b1, const float* __restrict__ g1,
                                                        const float* __restrict__ be1, bf16* __restrict__ out,
                                                        int64_t out_seq_stride, int r0, int r1) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[B_LDS];
  unsigned char* G = smem + B_OFF_G;
  unsigned char* Wt = smem + B_OFF_W;
  unsigned char* SV = smem + B_OFF_SV;
  float* RS = (float*)(smem + B_OFF_RS);
  float* WV = (float*)(smem + B_OFF_WV);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;  // 64 rows (t) x 128 output channels per wave
  const int s = blockIdx.y;
  const int t0 = r0 + blockIdx.x * BM;
  const float* src = wav + (int64_t)s * N;
  const unsigned char* W1b = (const unsigned char*)W1;

  // W1 DMA: a piece = 8 rows x 128 B; wave w fills pieces 8w..8w+7 of a 32-piece stage; lane ->
  // (row 8p + lane/8, physical chunk lane%8) holding logical chunk (lane%8) ^ bswz(row)
  uint32_t woff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = (w * 8 + i) * 8 + (lane >> 3);
    woff[i] = (uint32_t)(row * 2048 + bswz(row, lane & 7) * 8) * 2;
  }
  auto kbase = [](int q) {  // k-step q (0..31): phase r = q>>3, tap half h = (q>>2)&1, 64-channel group q&3
    return ((q >> 3) + 4 * ((q >> 2) & 1)) * 256 + (q & 3) * 64;
  };
  auto dma = [&](int q) {
    unsigned char* base = Wt + (q & 1) * BN * BROWB;
    const uint32_t kb = (uint32_t)kbase(q) * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(W1b + (woff[i] + kb)), (lds_void_t*)(base + (w * 8 + i) * 1024), 16, 0, 0);
  };

  // conv0 operand fragments of this wave (channel tiles 4w..4w+3) and folded ChannelNorm shifts
  chunk16 a0f[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a0f[j] = c0w[((4 * w + j) * 16 + (lane & 15)) * 4 + (lane >> 4)];
  float bet[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bet[j][e] = beta0[(4 * w + j) * 16 + 4 * (lane >> 4) + e];

  // the tile's waveform segment: samples 20*t0 - 13 + [0, WSEG) (zeros outside the signal)
  const int64_t xb = (int64_t)20 * t0 - 13;
  for (int i = tid; i < WSEG; i += 256) {
    const int64_t ix = xb + i;
    WV[i] = (ix >= 0 && ix < N) ? src[ix] : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // only the DMA ring uses vmcnt from here on
  dma(0);
  lds_barrier();

  f32x4 acc[8][4];  // [n tile][m tile] of C^T
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int r = 0; r < 4; ++r) {
    // ---------------- (a) split samples + ChannelNorm statistics of the phase positions (LDS only)
    if (tid < NPOS) {
      const int i = tid;
      const int p = 4 * (t0 + i) - 2 + r;
      const bool valid = i < GROWS && p >= 0 && p < L0;
      float sm[10];
#pragma unroll
      for (int k = 0; k < 10; ++k) sm[k] = WV[min(20 * i + 5 * r + k, WSEG - 1)];
      bf16 hi[10], lo[10];
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        hi[k] = (bf16)sm[k];
        lo[k] = (bf16)(sm[k] - (float)hi[k]);
      }
      bf16x8 v0 = {hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]};
      bf16x8 v1 = {hi[8], hi[9], lo[0], lo[1], lo[2], lo[3], lo[4], lo[5]};
      bf16x8 v2 = {lo[6], lo[7], lo[8], lo[9], hi[0], hi[1], hi[2], hi[3]};
      bf16x8 v3 = {hi[4], hi[5], hi[6], hi[7], hi[8], hi[9], (bf16)1.0f, (bf16)1.0f};
      unsigned char* row = SV + i * SVROW;
      *(bf16x8*)(row + 0) = v0;
      *(bf16x8*)(row + 16) = v1;
      *(bf16x8*)(row + 32) = v2;
      *(bf16x8*)(row + 48) = v3;
      float q = c0stat[C0Stat::BETA];
#pragma unroll
      for (int a = 0; a < 10; ++a) {
        float ga = 2.0f * c0stat[C0Stat::H + a];
#pragma unroll
        for (int b = 0; b < 10; ++b) ga = fmaf(c0stat[C0Stat::G + a * 10 + b], sm[b], ga);
        q = fmaf(ga, sm[a], q);
      }
      RS[i] = valid ? rsqrtf(fmaxf(q, 0.f) * (1.0f / 255.0f) + 1e-5f) : -1.0f;
    }
    lds_barrier();  // SV/RS ready; every wave done reading the previous phase's G

    // ---------------- (b) conv0 on the MFMA -> ChannelNorm/ReLU -> bf16 G image
#pragma unroll
    for (int pt = 0; pt < NPOS / 16; ++pt) {
      const int prow = pt * 16 + (lane & 15);
      const chunk16 bfr = *(const chunk16*)(SV + prow * SVROW + (lane >> 4) * 16);
      const float rs = RS[prow];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
        z = mfma_chunk<bf16>(a0f[j], bfr, z);
        if (prow < GROWS) {
          const int c = (4 * w + j) * 16 + 4 * (lane >> 4);
          bf16x4 o4;
#pragma unroll
          for (int e = 0; e < 4; ++e) o4[e] = (bf16)(rs < 0.f ? 0.f : fmaxf(fmaf(rs, z[e], bet[j][e]), 0.f));
          *(bf16x4*)(G + prow * GROWB + gswz(prow, c >> 3) * 16 + (c & 7) * 2) = o4;
        }
      }
    }
    lds_barrier();  // G ready

    // ---------------- (c) 8 k-steps of 64 over taps r (h = 0) and r + 4 (h = 1)
    for (int kq = 0; kq < 8; ++kq) {
      const int q = r * 8 + kq;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage q landed
      __builtin_amdgcn_s_barrier();                       // every wave's; stage q-1's buffer fully read
      __builtin_amdgcn_sched_barrier(0);
      if (q + 1 < 32) dma(q + 1);
      const int hh = kq >> 2, kk = kq & 3;
      const unsigned char* wb = Wt + (q & 1) * BN * BROWB;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        chunk16 gf[4], wf[8];
        const int c16 = kk * 8 + sub * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * 64 + i * 16 + (lane & 15) + hh;
          gf[i] = *(const chunk16*)(G + row * GROWB + gswz(row, c16) * 16);
        }
        const int cb = sub * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int row = wn * 128 + j * 16 + (lane & 15);
          wf[j] = *(const chunk16*)(wb + row * BROWB + bswz(row, cb) * 16);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[j][i] = mfma_chunk<bf16>(wf[j], gf[i], acc[j][i]);
      }
    }
  }

  // ---------------- epilogue: + b1, ChannelNorm (unbiased) over the 256 channels, ReLU, bf16
  // lane holds C[m = wm*64 + i*16 + lane%16][n = wn*128 + j*16 + (lane/16)*4 + e]
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // no DMA in flight; every wave done with the W1 stages (reused below)
  const int nb = wn * 128 + (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f32x4 b = *(const f32x4*)(b1 + nb + j * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] += b;
  }
  float* red = (float*)Wt;  // [BM][2 waves along N] (stride 4)
  float mean[4], rstd[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    if ((lane >> 4) == 0) red[(wm * 64 + i * 16 + (lane & 15)) * 4 + wn] = sum;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 pr = *(const f32x4*)(red + (wm * 64 + i * 16 + (lane & 15)) * 4);
    mean[i] = (pr[0] + pr[1]) * (1.0f / BN);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = acc[j][i][e] - mean[i];
        ss += d * d;
      }
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if ((lane >> 4) == 0) red[(wm * 64 + i * 16 + (lane & 15)) * 4 + wn] = ss;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 pr = *(const f32x4*)(red + (wm * 64 + i * 16 + (lane & 15)) * 4);
    rstd[i] = rsqrtf((pr[0] + pr[1]) * (1.0f / (BN - 1)) + 1e-5f);
  }
  bf16* obase = out + (int64_t)s * out_seq_stride;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f32x4 ga = *(const f32x4*)(g1 + nb + j * 16);
    const f32x4 be = *(const f32x4*)(be1 + nb + j * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + wm * 64 + i * 16 + (lane & 15);
      if (t >= r1) continue;
      f32x4 v = (acc[j][i] - mean[i]) * rstd[i] * ga + be;
      store4(obase + (int64_t)t * BN + nb + j * 16, fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f),
             fmaxf(v[3], 0.f));
    }
  }
}

}  // namespace

hipError_t launch_conv01(const float* wav, int S, int64_t N, int L0, int L1, const bf16* c0w, const float* c0stat,
                         const float* beta0, const bf16* W1, const float* b1, const float* g1, const float* be1,
                         bf16* out, int64_t out_seq_stride, hipStream_t st, int r0, int r1) {
  if (r1 < 0) r1 = L1;
  if (S <= 0 || L1 <= 0 || r0 < 0 || r1 > L1 || r0 >= r1) return hipErrorInvalidValue;
  dim3 grid((r1 - r0 + BM - 1) / BM, S);
  static const bool stamps = getenv("VAP_CONV01_STAMPS") != nullptr;
  static const int ver = getenv("VAP_CONV01_V1") ? 1 : (getenv("VAP_CONV01_V3") ? 3 : 2);
  if (ver == 1)
    hipLaunchKernelGGL(conv01_kernel, grid, dim3(512), 0, st, wav, N, L0, L1, (const chunk16*)c0w, c0stat, beta0, W1,
                       b1, g1, be1, out, out_seq_stride, r0, r1);
  else if (ver == 2 && !stamps)
    hipLaunchKernelGGL(conv01b_kernel<false>, grid, dim3(512), 0, st, wav, N, L0, (const chunk16*)c0w, c0stat, beta0, W1,
                       b1, g1, be1, out, out_seq_stride, r0, r1);
  else if (ver == 2)
    hipLaunchKernelGGL(conv01b_kernel<true>, grid, dim3(512), 0, st, wav, N, L0, (const chunk16*)c0w, c0stat, beta0, W1,
                       b1, g1, be1, out, out_seq_stride, r0, r1);
  else
    hipLaunchKernelGGL(conv01c_kernel, grid, dim3(256), 0, st, wav, N, L0, (const chunk16*)c0w, c0stat, beta0, W1, b1,
                       g1, be1, out, out_seq_stride, r0, r1);
  return hipGetLastError();
}

// diagnostics: copy the conv01 v2 phase stamps (8 sampled workgroups x 24) to host memory
hipError_t read_conv01_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_conv01_stamps), sizeof(g_conv01_stamps), 0, hipMemcpyDeviceToHost);
}
