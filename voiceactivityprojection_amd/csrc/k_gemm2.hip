// bf16 MFMA GEMM, 256 x 256 tiles, LDS-DMA staging (the bf16 perf path of launch_gemm).
//
// Same contract as gemm_kernel (k_gemm.hip): implicit-convolution A rows (lda may be < K, per
// sequence strides), W [N][K], fused bias / ChannelNorm | LayerNorm / ReLU | GELU / fp32 residual
// epilogue, bf16 or fp32 output.  Used for the CPC conv2..4 (k4 s2 implicit convs, K = 1024), the
// LSTM input projection, the downsample conv (+LN+GELU), FFN-down (+residual), combinator and heads.
//
// Structure (MI355X):
//   * 256 x 256 output tile per workgroup, 8 waves as 2 (M) x 4 (N), 128 x 64 outputs per wave:
//     W is re-read from L2 once per 256 rows (not per 128), A once per tile;
//   * K staged 32 deep (64-byte rows) by global_load_lds_dwordx4: 16 DMA pieces of 16 rows x 64 B
//     per operand and stage, 2 + 2 per wave, no VGPR staging.  The LDS image is lane-linear, the
//     XOR swizzle (conflict-free ds_read_b128 for 16 consecutive rows) is applied to the SOURCE
//     address and again on the fragment read;
//   * four 32 KiB stages, DMA three stages ahead (96 KiB in flight; raw s_barrier, counted vmcnt —
//     no __syncthreads, whose fence would drain them), and ping-pong scheduling of the two waves
//     that share each SIMD (one reads fragments while the other runs its MFMAs);
//   * operands swapped (C^T = W A^T) so a lane owns 4 consecutive columns of one row: 8-byte bf16 /
//     16-byte fp32 stores and residual loads, row statistics by a 16-lane-stride shuffle + LDS.
#include <cstdlib>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 32, ROWB = 64;  // BK bf16 = 64 B per staged row
constexpr int NST = 4;                                  // stages: 3 in flight while one computes
constexpr int STAGE = (BM + BN) * ROWB;                 // 32 KiB
typedef __attribute__((address_space(3))) void lds_void;

// 64-byte rows, 4 chunks: conflict-free ds_read_b128 for 16 consecutive rows x 4 chunks
VAP_DEV int swz(int row, int c) { return c ^ ((row >> 2) & 2); }

// diagnostics (VAP_GEMM2_STAMPS=1): waves 0 and 4 of workgroups 0, 64, .., 448 record s_memtime at
// k-steps 8..11: [LOAD start, fragments in, after LOAD barrier, MFMAs done, DMA wait done, after
// COMPUTE barrier] -> g_g2_stamps[wg][wave 0/4][4 k-steps][6]
__device__ unsigned long long g_g2_stamps[8][2][4][6];
// tile phases of the same sampled workgroups (wave 0): [0] start, [1] first stages landed, [2] k-loop
// done, [3] epilogue math done, [4] stores issued, [5] stores complete
__device__ unsigned long long g_g2_tile[8][6];

// ACT = g.act as a template parameter: a runtime branch between the activations over the 128 live
// accumulator registers made the compiler copy all of them at the merge and spill (scratch in the
// epilogue: 148-180 B per lane, written and read back once per tile)
template <typename TOut, bool ST, int ACT>
__global__ __launch_bounds__(512, 1) void gemm2_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int M = g.M_per_seq * g.n_seq;
  // XCD-aware tile order (1-D grid): blocks b, b + 8, .. share an XCD's L2 (round-robin dealing), so
  // the N / BN column tiles of one row tile go to consecutive slots of ONE XCD and its A rows are
  // fetched from HBM once instead of once per column tile
  const int ntn = g.N / BN;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int mt = (slot / ntn) * 8 + xcd;
  // c_pair (LSTM gate projection into the pair-recurrence layout): a tile is 16 steps x 16 sequences,
  // tile row r = sequence 16 pg + r % 16 at step 16 pt + r / 16
  const int ntb = g.c_pair ? (g.M_per_seq + 15) / 16 : 1;
  const int mtiles = g.c_pair ? (g.n_seq + 15) / 16 * ntb : (M + BM - 1) / BM;
  if (mt >= mtiles) return;  // padding block (whole workgroup, before any barrier)
  const int m0 = mt * BM, n0 = (slot % ntn) * BN;
  const int pg = mt / ntb, pt = mt - pg * ntb;
  const bf16* __restrict__ A = (const bf16*)g.A;
  const bf16* __restrict__ W = (const bf16*)g.W;
  const int samp = (ST && (mt & 63) == 0 && mt < 512 && n0 == 0 && (lane == 0) && (wave == 0 || wave == 4))
                       ? (int)(mt >> 6)
                       : -1;
  auto stamp = [&](int kt, int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (samp >= 0 && kt >= 8 && kt < 12) g_g2_stamps[samp][wave >> 2][kt - 8][k] = t;
    }
  };
  unsigned long long tst[6] = {};
  auto tstamp = [&](int k) {
    if constexpr (ST) {
      __builtin_amdgcn_sched_barrier(0);
      tst[k] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  tstamp(0);

  // DMA sources: a piece (one wave instruction, 1 KiB) = 16 rows x 64 B; wave w fills pieces 2w and
  // 2w+1 of each operand image; lane -> (row 16p + lane/4, physical chunk lane%4) holding logical
  // chunk (lane%4) ^ swz(row).  32-bit byte offsets from the uniform operand bases (saddr+voffset).
  uint32_t aoff[2], boff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 16 + (lane >> 2);
    const int c = swz(row, lane & 3);
    int s, t;
    if (g.c_pair) {
      s = pg * 16 + (row & 15);
      t = pt * 16 + (row >> 4);
      if (s >= g.n_seq || t >= g.M_per_seq) s = t = 0;  // tail rows: any valid row (never stored)
    } else {
      int m = m0 + row;
      m = m < M ? m : M - 1;  // tail rows: any valid row (never stored)
      s = m / g.M_per_seq;
      t = m - s * g.M_per_seq;
    }
    aoff[i] = (uint32_t)(((int64_t)s * g.a_seq_stride + (int64_t)t * g.lda + c * 8) * 2);
    boff[i] = (uint32_t)(((int64_t)(n0 + row) * g.K + c * 8) * 2);
  }
  const unsigned char* Ab = (const unsigned char*)A;
  const unsigned char* Wb = (const unsigned char*)W;
  // k-step order: with overlapping implicit-conv rows (lda < K, K = taps x 256), tap-inner order
  // (256-channel block outer) makes row t's tap j+2 -- the same input row as row t+1's tap j -- be
  // read two k-steps later instead of 16, while it is still in L2 (sequential order fetched the
  // input twice from HBM).  Only the summation order changes.
  const int taps = g.lda < g.K && g.K % 256 == 0 ? g.K / 256 : 1;
  auto koff = [&](int kt) -> uint32_t {  // byte offset of k-step kt within a row
    if (taps == 1) return (uint32_t)kt * ROWB;
    const int cb = kt / taps, tap = kt - cb * taps;
    return (uint32_t)(tap * 256 + cb * BK) * 2;
  };
  auto dma = [&](int kt) {
    unsigned char* base = smem + (kt % NST) * STAGE;
    const uint32_t kb = koff(kt);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(Ab + (aoff[i] + kb)), (lds_void*)(base + (wave * 2 + i) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(Wb + (boff[i] + kb)), (lds_void*)(base + BM * ROWB + (wave * 2 + i) * 1024),
                                       16, 0, 0);
  };

  f32x4 acc[4][8];  // [n tile][m tile] of C^T
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (row-dependent part; the chunk varies with the k half)
  const int fr = lane & 15, fc = lane >> 4;
  const int nk = g.K / BK;
  // Ping-pong: waves 0-3 and 4-7 (one of each per SIMD) run half a k-step apart.  Every k-step is
  // a LOAD phase (issue the DMA three stages ahead, read this stage's fragments) and a COMPUTE phase
  // (32 MFMAs), each closed by a workgroup barrier; group 1 enters one barrier late, so on every
  // SIMD one wave's MFMAs overlap the other wave's LDS reads.
  //   RAW: a wave waits (counted vmcnt) for its own DMA of stage t+1 before the barrier that precedes
  //        any wave's first read of stage t+1: group 0 at the end of COMPUTE t, group 1 (one barrier
  //        behind) at the end of LOAD t, which meets group 0's end-of-COMPUTE barrier.
  //   WAR: stage t+3 overwrites stage t-1's buffer; its last reads (group 1's LOAD t-1) retire with
  //        lgkmcnt(0) before the barrier that precedes group 0's LOAD t.
  const int grp = wave >> 2;
#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nk) dma(p);
  if (nk >= 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (nk == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  tstamp(1);
  if (grp == 1) __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    // ---- LOAD
    __builtin_amdgcn_sched_barrier(0);
    stamp(kt, 0);
    if (kt + NST - 1 < nk) dma(kt + NST - 1);
    const unsigned char* abase = smem + (kt % NST) * STAGE;
    const unsigned char* bbase = abase + BM * ROWB;
    chunk16 wf[4], af[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + j * 16 + fr;
      wf[j] = *(const chunk16*)(bbase + row * ROWB + swz(row, fc) * 16);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wm * 128 + i * 16 + fr;
      af[i] = *(const chunk16*)(abase + row * ROWB + swz(row, fc) * 16);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // group 1's own DMA of stage kt+1 must land before THIS barrier: it is the one after which group 0
    // reads stage kt+1 (group 1's own end-of-COMPUTE wait comes one barrier later; a late piece was
    // read stale by a group-0 wave)
    if (grp == 1) {
      if (kt + 3 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    stamp(kt, 1);
    __builtin_amdgcn_s_barrier();
    stamp(kt, 2);
    // ---- COMPUTE
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = mfma_chunk<bf16>(wf[j], af[i], acc[j][i]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    stamp(kt, 3);
    // own DMA of stage kt+1 landed: newer DMAs are those of stages kt+2 and kt+3 (4 each, if issued)
    if (kt + 3 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(kt, 4);
    __builtin_amdgcn_s_barrier();
    stamp(kt, 5);
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  tstamp(2);

  // ---------------------------------------------------------------- epilogue
  // lane holds C[m = m0 + wm*128 + i*16 + fr][n = n0 + wn*64 + j*16 + fc*4 + r]
  const int nb = n0 + wn * 64 + fc * 4;
  if (g.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 b = *(const f32x4*)(g.bias + nb + j * 16);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] += b;
    }
  }
  if (g.norm) {
    __syncthreads();  // all DMA retired (vmcnt(0) above) and every wave done reading the stages
    float* red = (float*)smem;  // [BM][4 waves along N]
    float mean[8], rstd[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) s += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (fc == 0) red[(wm * 128 + i * 16 + fr) * 4 + wn] = s;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 p = *(const f32x4*)(red + (wm * 128 + i * 16 + fr) * 4);
      mean[i] = (p[0] + p[1] + p[2] + p[3]) * (1.0f / BN);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[j][i][r] - mean[i];
          s += d * d;
        }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (fc == 0) red[(wm * 128 + i * 16 + fr) * 4 + wn] = s;
    }
    __syncthreads();
    const float inv_n = g.norm == 1 ? 1.0f / (BN - 1) : 1.0f / BN;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 p = *(const f32x4*)(red + (wm * 128 + i * 16 + fr) * 4);
      rstd[i] = rsqrtf((p[0] + p[1] + p[2] + p[3]) * inv_n + g.eps);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 ga = *(const f32x4*)(g.gamma + nb + j * 16);
      const f32x4 be = *(const f32x4*)(g.beta + nb + j * 16);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = (acc[j][i] - mean[i]) * rstd[i] * ga + be;
    }
  }
  if constexpr (ACT == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[j][i][r] = fmaxf(acc[j][i][r], 0.f);
  } else if constexpr (ACT == 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f32x2 lo = gelu_fast2((f32x2){acc[j][i][0], acc[j][i][1]});
        const f32x2 hi = gelu_fast2((f32x2){acc[j][i][2], acc[j][i][3]});
        acc[j][i] = f32x4{lo[0], lo[1], hi[0], hi[1]};
      }
  }
  tstamp(3);
  TOut* __restrict__ C = (TOut*)g.C;
  if (g.c_pair) {  // gate rows into the pair-recurrence layout: the lane's 4 column blocks are the 4 gates of
                   // units 16ub + 4fc .. +3 (W rows in gx_wrow order), i.e. one whole record of 2 x 16 bytes
    const int ub = (n0 + wn * 64) >> 6;
    const int s = pg * 16 + fr;
    if (s < g.n_seq) {
      const int gsq = g.c_s0 + s;
      const int64_t lo = (int64_t)((fc * 16 + (gsq & 15)) * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int t = pt * 16 + wm * 8 + i;
        if (t >= g.M_per_seq) continue;
        int sl = g.c_t0 + t;
        sl = sl >= g.c_tn ? sl - g.c_tn : sl;
        bf16* rec = (bf16*)C + gx_pair_block(gsq >> 4, sl, ub, g.c_tn) + lo;
        const u32x2 a0 = pack_bf16x4(acc[0][i][0], acc[0][i][1], acc[0][i][2], acc[0][i][3]);
        const u32x2 a1 = pack_bf16x4(acc[1][i][0], acc[1][i][1], acc[1][i][2], acc[1][i][3]);
        const u32x2 a2 = pack_bf16x4(acc[2][i][0], acc[2][i][1], acc[2][i][2], acc[2][i][3]);
        const u32x2 a3 = pack_bf16x4(acc[3][i][0], acc[3][i][1], acc[3][i][2], acc[3][i][3]);
        // streaming (nt) stores: the recurrence reads these rows much later (the buffer is 4 MiB per 16
        // sequences per 1000 steps, far beyond L2); plain stores evicted W and A rows from L2 (FETCH
        // 235 -> 138 MB per 128-sequence launch, 1.79x -> 1.06x algorithmic; lstm_proj 0.286 -> 0.272 ms)
        __builtin_nontemporal_store(u32x4{a0[0], a0[1], a1[0], a1[1]}, (u32x4*)rec);
        __builtin_nontemporal_store(u32x4{a2[0], a2[1], a3[0], a3[1]}, (u32x4*)(rec + 512));
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + fr;
    if (m >= M) continue;
    const int s = m / g.M_per_seq, t = m - s * g.M_per_seq;
    TOut* crow = C + (int64_t)s * g.c_seq_stride + (int64_t)t * g.ldc + nb;
    const float* arow = g.add ? g.add + (int64_t)s * g.add_seq_stride + (int64_t)t * g.ld_add + nb : nullptr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 v = acc[j][i];
      if (arow) v += *(const f32x4*)(arow + j * 16);
      store4(crow + j * 16, v[0], v[1], v[2], v[3]);
    }
  }
  if constexpr (ST) {
    tstamp(4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tstamp(5);
    if (samp >= 0 && wave == 0)
      for (int k = 0; k < 6; ++k) g_g2_tile[samp][k] = tst[k];
  }
}

}  // namespace

template <typename TOut>
hipError_t launch_gemm2(const GemmArgs& g, hipStream_t st) {
  const int M = g.M_per_seq * g.n_seq;
  if (g.K % BK != 0 || g.N % BN != 0 || M <= 0) return hipErrorInvalidValue;
  if (g.norm && g.N != BN) return hipErrorInvalidValue;
  // 16-byte alignment of every DMA source / epilogue vector access
  if (g.lda % 8 || g.a_seq_stride % 8 || g.ldc % 4 || g.c_seq_stride % 4 || (g.add && (g.ld_add % 4 || g.add_seq_stride % 4)))
    return hipErrorInvalidValue;
  if (g.c_pair && (sizeof(TOut) != 2 || g.N != 1024 || g.norm || g.act || g.add || g.c_tn <= 0 || g.c_t0 < 0 ||
                   g.c_t0 >= g.c_tn || g.M_per_seq > g.c_tn || g.c_s0 < 0))
    return hipErrorInvalidValue;
  const int mtiles = g.c_pair ? (g.n_seq + 15) / 16 * ((g.M_per_seq + 15) / 16) : (M + BM - 1) / BM;
  const dim3 grid((unsigned)((mtiles + 7) / 8 * 8 * (g.N / BN)));  // XCD-aware 1-D order (see the kernel)
  static const bool stamps = getenv("VAP_GEMM2_STAMPS") != nullptr;
  if (g.act < 0 || g.act > 2) return hipErrorInvalidValue;
  auto go = [&](auto stc) {
    constexpr bool S_ = decltype(stc)::value;
    if (g.act == 1) hipLaunchKernelGGL((gemm2_kernel<TOut, S_, 1>), grid, dim3(512), 0, st, g);
    else if (g.act == 2) hipLaunchKernelGGL((gemm2_kernel<TOut, S_, 2>), grid, dim3(512), 0, st, g);
    else hipLaunchKernelGGL((gemm2_kernel<TOut, S_, 0>), grid, dim3(512), 0, st, g);
  };
  if (stamps) go(std::true_type{});
  else go(std::false_type{});
  return hipGetLastError();
}

// diagnostics: copy the gemm2 k-step stamps (8 x 2 x 4 x 6) to host memory
hipError_t read_gemm2_stamps(unsigned long long* out) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_g2_stamps), sizeof(g_g2_stamps), 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbol(out + 8 * 2 * 4 * 6, HIP_SYMBOL(g_g2_tile), sizeof(g_g2_tile), 0, hipMemcpyDeviceToHost);
}

template hipError_t launch_gemm2<bf16>(const GemmArgs&, hipStream_t);
template hipError_t launch_gemm2<float>(const GemmArgs&, hipStream_t);
