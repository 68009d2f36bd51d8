// Fused transformer FFN block (bf16 perf path):
//
//   x += W2 . GELU(W1 . LayerNorm(x))          (modules.py:9-21 ffn_block, TransformerLayer :273-275)
//
// per 64-row panel, with the 768-wide hidden activation kept in LDS: the LayerNorm'd panel
// (32 KiB bf16) and the GELU'd hidden (64 x 768 bf16 = 96 KiB) never touch HBM, where the
// unfused pair wrote and re-read 2 x 49 MB per 32k rows.  W1 [768][256] and then W2 [256][768] stream
// through one register-prefetched, double-buffered LDS stage ring (256 rows x 32 k, 32 KiB): 24
// k-steps of the up-projection (3 N tiles of 256) followed by 24 k-steps of the down-projection.
// Operands are swapped (C^T = W . A^T) so a lane owns 4 consecutive columns of a row: 8-byte bf16
// writes into the hidden image, 16-byte residual reads / fp32 stores.
// LDS 160 KiB -> one workgroup (4 waves, one per SIMD) per CU.
#include "vap_common.h"
#include "vap_kernels.h"

namespace {

constexpr int BM = 64, D = 256, DF = 768;
constexpr int PROWB = D * 2;    // LN panel row: 512 B
constexpr int HROWB = DF * 2;   // hidden row: 1536 B
constexpr int BK = 32, WROWB = BK * 2;
constexpr int OFF_H = BM * PROWB;             // 32 KiB
constexpr int OFF_W = OFF_H + BM * HROWB;     // + 96 KiB
constexpr int LDS_BYTES = OFF_W + 2 * D * WROWB;  // + 32 KiB = 160 KiB
constexpr int NQ1 = (DF / D) * (D / BK);      // 24 up-projection k-steps
constexpr int NQ = NQ1 + DF / BK;             // + 24 down-projection k-steps
constexpr int NPF = 4;

VAP_DEV int pswz(int row, int c16) { return c16 ^ (row & 15); }              // 32 chunks per panel row
VAP_DEV int hswz(int row, int c16) { return c16 ^ (row & 15); }              // 96 chunks per hidden row
VAP_DEV int wswz(int row, int c) { return c ^ ((row >> 2) & 2); }            // 4 chunks per W row

__global__ __launch_bounds__(256, 1) void ffn_kernel(FfnArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  unsigned char* P = smem;
  unsigned char* Hh = smem + OFF_H;
  unsigned char* Wt = smem + OFF_W;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * BM;
  const bf16* __restrict__ W1 = (const bf16*)g.W1;
  const bf16* __restrict__ W2 = (const bf16*)g.W2;
  auto xoff = [&](int m) -> int64_t {  // element offset of row m of x
    if (g.rows_per_seq == 0) return (int64_t)m * D;
    const int sq = m / g.rows_per_seq;
    return (int64_t)sq * g.x_seq + (int64_t)(m - sq * g.rows_per_seq) * D;
  };

  // W stream: k-step q < 24: W1 rows nt*256 + row, k = kq*32; q >= 24: W2 rows row, k = (q-24)*32
  chunk16 rb[NPF][4];
  auto gload = [&](int q, chunk16* r) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * 256, row = id >> 2, c = id & 3;
      const bf16* src = q < NQ1 ? W1 + (int64_t)((q >> 3) * D + row) * D + (q & 7) * BK + c * 8
                                : W2 + (int64_t)row * DF + (q - NQ1) * BK + c * 8;
      r[i] = *(const chunk16*)src;
    }
  };
  auto lstore = [&](int buf, const chunk16* r) {
    unsigned char* base = Wt + buf * D * WROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * 256, row = id >> 2, c = id & 3;
      *(chunk16*)(base + row * WROWB + wswz(row, c) * 16) = r[i];
    }
  };
#pragma unroll
  for (int p = 0; p < NPF; ++p) gload(p, rb[p]);

  // ------------------------------------------------------------ LayerNorm(x) panel -> LDS (bf16)
  // (the coalesced fp32 row load of k_rowpanel.hip: 16 lanes read 256 contiguous bytes of a row)
  {
    const int r4 = lane >> 4, cc = lane & 15;
    f32x4 v[4][4];
#pragma unroll
    for (int set = 0; set < 4; ++set) {
      const int m = m0 + w * 16 + set * 4 + r4;
      const float* src = g.x + xoff(m < g.M ? m : 0) + cc * 4;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) v[set][jj] = m < g.M ? *(const f32x4*)(src + jj * 64) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 ga[4], be[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      ga[jj] = *(const f32x4*)(g.gamma + jj * 64 + cc * 4);
      be[jj] = *(const f32x4*)(g.beta + jj * 64 + cc * 4);
    }
#pragma unroll
    for (int set = 0; set < 4; ++set) {
      float sum = 0.f;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) sum += v[set][jj][0] + v[set][jj][1] + v[set][jj][2] + v[set][jj][3];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
      const float mean = sum * (1.0f / D);
      float ss = 0.f;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v[set][jj] -= mean;
        ss += v[set][jj][0] * v[set][jj][0] + v[set][jj][1] * v[set][jj][1] + v[set][jj][2] * v[set][jj][2] +
              v[set][jj][3] * v[set][jj][3];
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) ss += __shfl_xor(ss, o, 64);
      const float rstd = rsqrtf(ss * (1.0f / D) + g.eps);
      const int row = w * 16 + set * 4 + r4;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const f32x4 y = v[set][jj] * rstd * ga[jj] + be[jj];
        const bf16x4 b = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
        *(bf16x4*)(P + row * PROWB + pswz(row, jj * 8 + (cc >> 1)) * 16 + (cc & 1) * 8) = b;
      }
    }
  }
  lstore(0, rb[0]);
  __syncthreads();

  // ------------------------------------------------------------ 48 k-steps: 3 x 8 up, 24 down
  f32x4 acc[4][4];  // [n tile 16 of the wave's 64 columns][m tile 16] of C^T
  for (int q0 = 0; q0 < NQ; q0 += NPF) {
#pragma unroll
    for (int p = 0; p < NPF; ++p) {
      const int q = q0 + p;
      const bool up = q < NQ1;
      const int kq = up ? (q & 7) : q - NQ1;  // k-step within the current GEMM
      if (kq == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      const unsigned char* wb = Wt + (q & 1) * D * WROWB;
      chunk16 wf[4], af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = w * 64 + i * 16 + (lane & 15);
        wf[i] = *(const chunk16*)(wb + row * WROWB + wswz(row, lane >> 4) * 16);
      }
      const int ca = kq * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = j * 16 + (lane & 15);
        af[j] = up ? *(const chunk16*)(P + row * PROWB + pswz(row, ca) * 16)
                   : *(const chunk16*)(Hh + row * HROWB + hswz(row, ca) * 16);
      }
      if (q + NPF < NQ) gload(q + NPF, rb[p]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_chunk<bf16>(wf[i], af[j], acc[i][j]);
      if (q + 1 < NQ) lstore((q + 1) & 1, rb[(p + 1) % NPF]);
      if (up && kq == 7) {
        // up-projection N tile done: GELU -> bf16 hidden columns nt*256 + w*64 + i*16 + (lane/16)*4
        const int nt = q >> 3;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = nt * D + w * 64 + i * 16 + (lane >> 4) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = j * 16 + (lane & 15);
            const f32x4 a = acc[i][j];
            const bf16x4 b = {(bf16)gelu_erf(a[0]), (bf16)gelu_erf(a[1]), (bf16)gelu_erf(a[2]), (bf16)gelu_erf(a[3])};
            *(bf16x4*)(Hh + row * HROWB + hswz(row, n >> 3) * 16 + ((n >> 2) & 1) * 8) = b;
          }
        }
      }
      if (!up && q == NQ - 1) {
        // down-projection done: x[m][n .. n+3] += acc  (fp32 residual, in place)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = m0 + j * 16 + (lane & 15);
          if (m >= g.M) continue;
          float* xr = g.x + xoff(m);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = w * 64 + i * 16 + (lane >> 4) * 4;
            f32x4 v = *(const f32x4*)(xr + n);
            v += acc[i][j];
            *(f32x4*)(xr + n) = v;
          }
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace

hipError_t launch_ffn(const FfnArgs& g, hipStream_t st) {
  if (g.M <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ffn_kernel, dim3((g.M + BM - 1) / BM), dim3(256), 0, st, g);
  return hipGetLastError();
}
