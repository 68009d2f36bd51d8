// Fused transformer FFN block (bf16 perf path):
//
//   x += W2 . GELU(W1 . LayerNorm(x))          (modules.py:9-21 ffn_block, TransformerLayer :273-275)
//
// per 64-row panel with the 768-wide hidden activation kept in LDS: the LayerNorm'd panel (32 KiB
// bf16) and the GELU'd hidden (64 x 768 bf16 = 96 KiB) never touch HBM, where the unfused pair
// (row-panel FFN-up + GEMM FFN-down) wrote and re-read 2 x 49 MB per 32k rows and read x twice.
//
// One workgroup of 8 waves (two per SIMD) per CU.  Both GEMMs take their weight operand straight
// from L2 into registers in the packed projection layout (k_misc.hip pack_rowpanel: one wave's
// 16-row fragment of a 32-deep k-step is 1 KiB contiguous), so the only LDS traffic is the
// activation operand and no k-loop needs a barrier:
//   FFN-up   (K 256, N 768): wave w owns hidden columns w*96 .. +95 (6 fragments x 4 row tiles),
//            8 k-steps, W1 fragments prefetched 2 steps ahead;  GELU -> bf16 -> hidden image.
//   FFN-down (K 768, N 256): wave w owns output columns w*32 .. +31 (2 fragments x 4 row tiles),
//            24 k-steps, W2 prefetched 4 steps ahead, hidden fragments double-buffered in
//            registers; the residual rows are prefetched when the loop starts.
// Every wave reads a distinct slice of W1 and W2, so each workgroup streams each weight once.
// Operands are swapped (C^T = W . A^T): a lane owns 4 consecutive columns of one row.
#include <cstdlib>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

constexpr int BM = 64, D = 256, DF = 768;
constexpr int PROWB = D * 2;                  // LN panel row: 512 B (32 chunks)
constexpr int HROWB = DF * 2;                 // hidden row: 1536 B (96 chunks)
// MT row tiles of 16 per workgroup (BM = 16 MT rows): LN panel 512 B + hidden 1536 B per row
template <int MT> constexpr int ffn_lds() { return MT * 16 * (PROWB + HROWB); }  // MT 4: 128 KiB, 5: 160 KiB
constexpr int NF1 = 6, NF2 = 2;               // weight fragments per wave: up / down
constexpr int KS1 = D / 32, KS2 = DF / 32;    // k-steps: 8 / 24
constexpr int NPF1 = 2, NPF2 = 4;             // weight prefetch depth (k-steps)

// 16-B chunk c of row `row`: XOR with row%16 spreads the 16 rows of an MFMA fragment read over
// 16 distinct bank groups (rows are 512 / 1536 B = 0 mod 256 B apart)
VAP_DEV int xswz(int row, int c) { return c ^ (row & 15); }

// diagnostics (VAP_FFN_STAMPS=1): wave 0 of workgroups 0, 64, .., 448 records s_memtime at [0] start,
// [1] LN panel written, [2] after the barrier, [3 + ks] FFN-up k-step ks (8), [11] up done, [12] GELU
// written, [13] after the barrier, [14 + ks/4] FFN-down k-steps 0, 4, .., 20, [20] stores issued,
// [21] stores done; [22] / [23] s_memrealtime (100 MHz) at start / end
__device__ unsigned long long g_ffn_stamps[8][24];
__device__ unsigned long long g_ffn_wall[1024][2];  // every workgroup < 1024: realtime start / end

template <bool ST, int MT>
__global__ __launch_bounds__(512, 1) void ffn_kernel(FfnArgs g) {
  constexpr int BMt = MT * 16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[ffn_lds<MT>()];
  unsigned char* P = smem;
  unsigned char* Hh = smem + BMt * PROWB;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * BMt;
  const bf16* __restrict__ W1 = (const bf16*)g.W1;
  const bf16* __restrict__ W2 = (const bf16*)g.W2;
  const int samp = (ST && (blockIdx.x & 63) == 0 && blockIdx.x < 512 && tid == 0) ? (int)(blockIdx.x >> 6) : -1;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (samp >= 0) g_ffn_stamps[samp][k] = t;
    }
  };
  stamp(0);
  if constexpr (ST) {
    if (samp >= 0) g_ffn_stamps[samp][22] = __builtin_amdgcn_s_memrealtime();  // 100 MHz wall clock
    if (tid == 0 && blockIdx.x < 1024) g_ffn_wall[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
  }
  auto xoff = [&](int m) -> int64_t {  // element offset of row m of x
    if (g.rows_per_seq == 0) return (int64_t)m * D;
    const int sq = m / g.rows_per_seq;
    return (int64_t)sq * g.x_seq + (int64_t)(m - sq * g.rows_per_seq) * D;
  };

  // ------------------------------------------------------------ LayerNorm(x) panel -> LDS (bf16)
  // wave w: rows w*8 .. w*8+7 as 2 sets of 4; a 16-lane group reads 256 contiguous bytes of its row
  // per load.  Loads are unconditional (clamped row + select): a load under a branch gets its own
  // s_waitcnt and serialises the panel.
  // 4-row sets s = w, w + 8, ... (BM / 4 sets over the 8 waves)
  constexpr int NSET = (BMt / 4 + 7) / 8;
  {
    const int r4 = lane >> 4, cc = lane & 15;
    f32x4 v[NSET][4];
#pragma unroll
    for (int set = 0; set < NSET; ++set) {
      const int m = m0 + (w + set * 8) * 4 + r4;
      const float* src = g.x + xoff(m < g.M ? m : g.M - 1) + cc * 4;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) v[set][jj] = *(const f32x4*)(src + jj * 64);
    }
    f32x4 ga[4], be[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      ga[jj] = *(const f32x4*)(g.gamma + jj * 64 + cc * 4);
      be[jj] = *(const f32x4*)(g.beta + jj * 64 + cc * 4);
    }
#pragma unroll
    for (int set = 0; set < NSET; ++set) {
      if (w + set * 8 >= BMt / 4) break;
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
      const int row = (w + set * 8) * 4 + r4;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {  // rows >= M hold LN(row M-1): computed, never stored
        const f32x4 y = v[set][jj] * rstd * ga[jj] + be[jj];
        const bf16x4 b = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
        *(bf16x4*)(P + row * PROWB + xswz(row, jj * 8 + (cc >> 1)) * 16 + (cc & 1) * 8) = b;
      }
    }
  }

  // ------------------------------------------------------------ FFN-up: 8 k-steps, N 768
  // fragment i of wave w = hidden rows of W1 (w*6 + i)*16 .. +15 = row group (w*6+i) of the packed
  // layout: N tile (w*6+i)/16, group (w*6+i)%16
  auto w1load = [&](int ks, chunk16* r) {
#pragma unroll
    for (int i = 0; i < NF1; ++i) {
      const int gg = w * NF1 + i;
      r[i] = *(const chunk16*)(W1 + ((((int64_t)(gg >> 4) * KS1 + ks) * 16 + (gg & 15)) * 64 + lane) * 8);
    }
  };
  chunk16 wb1[NPF1][NF1];
#pragma unroll
  for (int p = 0; p < NPF1; ++p) w1load(p, wb1[p]);
  stamp(1);
  __syncthreads();  // LN panel complete
  stamp(2);

  f32x4 acc1[NF1][MT];
#pragma unroll
  for (int i = 0; i < NF1; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks) {
    stamp(3 + ks);
    chunk16 af[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int row = j * 16 + (lane & 15);
      af[j] = *(const chunk16*)(P + row * PROWB + xswz(row, ks * 4 + (lane >> 4)) * 16);
    }
    chunk16* wf = wb1[ks % NPF1];
#pragma unroll
    for (int i = 0; i < NF1; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc1[i][j] = mfma_chunk<bf16>(wf[i], af[j], acc1[i][j]);
    // unconditional refill (the tail reloads the last step): conditional loads make the compiler's
    // vmcnt bookkeeping drain the whole prefetch
    w1load(ks + NPF1 < KS1 ? ks + NPF1 : KS1 - 1, wf);
  }

  stamp(11);
  // W2 prefetch and the residual rows go out before the GELU epilogue so their latency hides
  // behind it.  fragment i of wave w = output rows of W2 (w*2+i)*16 .. +15 (one N tile of 256)
  auto w2load = [&](int ks, chunk16* r) {
#pragma unroll
    for (int i = 0; i < NF2; ++i)
      r[i] = *(const chunk16*)(W2 + ((((int64_t)ks) * 16 + w * NF2 + i) * 64 + lane) * 8);
  };
  chunk16 wb2[NPF2][NF2];
#pragma unroll
  for (int p = 0; p < NPF2; ++p) w2load(p, wb2[p]);
  // this lane's 4 rows (j*16 + lane%16) as byte offsets from the panel's first row of x; rows >= M
  // are out of range for the buffer resource: their residual reads return 0, their stores drop
  const int64_t xbase = xoff(m0);
  uint32_t xrow[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = m0 + j * 16 + (lane & 15);
    xrow[j] = m < g.M ? (uint32_t)((xoff(m) - xbase) * 4) : 0x80000000u;
  }
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(g.x + xbase, 0x7FFFFFF0u);
  f32x4 res[NF2][MT];
#pragma unroll
  for (int i = 0; i < NF2; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j)
      res[i][j] = __builtin_bit_cast(f32x4, buf_load16(rx, xrow[j] + (uint32_t)(w * 32 + i * 16 + (lane >> 4) * 4) * 4u, 0));

  // GELU -> bf16 hidden image: lane holds hidden columns n .. n+3 of row j*16 + lane%16
#pragma unroll
  for (int i = 0; i < NF1; ++i) {
    const int n = (w * NF1 + i) * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int row = j * 16 + (lane & 15);
      const f32x4 a = acc1[i][j];
      const f32x2 lo = gelu_fast2((f32x2){a[0], a[1]}), hi = gelu_fast2((f32x2){a[2], a[3]});
      const bf16x4 b = {(bf16)lo[0], (bf16)lo[1], (bf16)hi[0], (bf16)hi[1]};
      *(bf16x4*)(Hh + row * HROWB + xswz(row, n >> 3) * 16 + ((n >> 2) & 1) * 8) = b;
    }
  }
  stamp(12);
  __syncthreads();  // hidden complete
  stamp(13);

  // ------------------------------------------------------------ FFN-down: 24 k-steps, N 256
  f32x4 acc2[NF2][MT];
#pragma unroll
  for (int i = 0; i < NF2; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto hread = [&](int ks, chunk16* af) {
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int row = j * 16 + (lane & 15);
      af[j] = *(const chunk16*)(Hh + row * HROWB + xswz(row, ks * 4 + (lane >> 4)) * 16);
    }
  };
  chunk16 ha[2][MT];
  hread(0, ha[0]);
#pragma unroll
  for (int ks = 0; ks < KS2; ++ks) {
    if (ks % 4 == 0) stamp(14 + ks / 4);
    if (ks + 1 < KS2) hread(ks + 1, ha[(ks + 1) & 1]);  // static condition (loop fully unrolled)
    chunk16* wf = wb2[ks % NPF2];
#pragma unroll
    for (int i = 0; i < NF2; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc2[i][j] = mfma_chunk<bf16>(wf[i], ha[ks & 1][j], acc2[i][j]);
    w2load(ks + NPF2 < KS2 ? ks + NPF2 : KS2 - 1, wf);
  }

  // x[m][n .. n+3] += acc  (fp32 residual in place; branch-free buffer stores)
#pragma unroll
  for (int i = 0; i < NF2; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const f32x4 v = res[i][j] + acc2[i][j];
      buf_store16_wt(rx, xrow[j] + (uint32_t)(w * 32 + i * 16 + (lane >> 4) * 4) * 4u, __builtin_bit_cast(u32x4, v));
    }
  if constexpr (ST) {
    stamp(20);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(21);
    if (samp >= 0) g_ffn_stamps[samp][23] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && blockIdx.x < 1024) g_ffn_wall[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
  }
}

}  // namespace

hipError_t launch_ffn(const FfnArgs& g, hipStream_t st) {
  if (g.M <= 0 || g.rows_per_seq < 0) return hipErrorInvalidValue;
  // 64-row panels; VAP_FFN_MT=5: 80-row panels (the whole 160 KiB of LDS), measured equal on the
  // bench (400 workgroups instead of 500 over the 248 CUs the concurrent LSTM leaves)
  static const int mt = getenv("VAP_FFN_MT") ? atoi(getenv("VAP_FFN_MT")) : 4;
  const int bm = (mt == 4 ? 4 : 5) * 16;
  // a panel's rows must lie within the 2 GiB a buffer offset reaches from its first row
  const int64_t span = g.rows_per_seq ? (bm / g.rows_per_seq + 2) * g.x_seq + (int64_t)bm * D : (int64_t)bm * D;
  if (span * 4 >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
  static const bool stamps = getenv("VAP_FFN_STAMPS") != nullptr;
  const dim3 grid((g.M + bm - 1) / bm);
  if (mt == 4) {
    if (stamps) hipLaunchKernelGGL((ffn_kernel<true, 4>), grid, dim3(512), 0, st, g);
    else hipLaunchKernelGGL((ffn_kernel<false, 4>), grid, dim3(512), 0, st, g);
  } else {
    if (stamps) hipLaunchKernelGGL((ffn_kernel<true, 5>), grid, dim3(512), 0, st, g);
    else hipLaunchKernelGGL((ffn_kernel<false, 5>), grid, dim3(512), 0, st, g);
  }
  return hipGetLastError();
}

// diagnostics: copy the FFN stamps (8 sampled workgroups x 24) to host memory
// (8 x 24 sampled phase stamps, then 1024 x 2 per-workgroup wall-clock start / end)
hipError_t read_ffn_stamps(unsigned long long* out) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ffn_stamps), sizeof(g_ffn_stamps), 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbol(out + 8 * 24, HIP_SYMBOL(g_ffn_wall), sizeof(g_ffn_wall), 0, hipMemcpyDeviceToHost);
}
