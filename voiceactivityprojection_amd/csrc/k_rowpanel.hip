// Row-panel GEMM for the transformer projections (bf16 perf mode), K = 256.
//
//   C[m, n] = epi( sum_k A'[m, k] W[n, k] ),   A' = LayerNorm(x[m]) | x[m] (fp32 -> bf16) | A[m] (bf16)
//
// Reference ops: the pre-LN TransformerLayer projections (vap/modules.py:246-275): LN_sa -> Q/K/V,
// raw src -> cross K/V, LN_src -> cross Q, attention output -> proj (+ residual), LN_ff -> FFN up
// (GELU).  K = dim = 256, so a 64-row A panel (32 KiB bf16) stays resident in LDS while EVERY
// 256-wide N tile of W streams past it: the activation is read once (not once per N tile) and the
// LayerNorm is computed while the panel is loaded (no LN kernel, no normalised copy in HBM).
// Operands are swapped (C^T[n][m] = W[n] . A[m]) so each lane owns 4 consecutive outputs of one
// row: 8-byte bf16 / 16-byte fp32 stores, 16-byte residual reads.
#include <cstdlib>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

// 64-row panels, 4 waves, W streamed in 32-deep k-steps: 64 KiB LDS -> two workgroups per CU, so
// one workgroup's panel load / stores overlap the other's MFMAs (a single resident workgroup
// serialises load -> compute -> store and leaves HBM or the matrix pipes idle).
constexpr int BM = 64, BN = 256, KP = 256, PROWB = KP * 2;  // A panel row: 512 B
constexpr int BK = 32, WROWB = BK * 2;                      // W staging row: 64 B
constexpr int OFF_W = BM * PROWB;                           // 32 KiB
constexpr int LDS_BYTES = OFF_W + 2 * BN * WROWB;           // + 32 KiB
constexpr int KSTEPS = KP / BK;                             // 8 per N tile
constexpr int NPF = 4;                                      // W prefetch depth (k-steps)

VAP_DEV int pswz(int row, int c16) { return c16 ^ (row & 15); }
VAP_DEV int wswz(int row, int c) { return c ^ ((row >> 2) & 2); }  // 64-B rows: b128 reads + writes conflict-free

// WD = false: W k-tiles staged through a double-buffered LDS ring (one barrier per k-step).
// WD = true:  every wave loads its own W fragments (its 64 columns = 64 W rows) straight from L2
//             into registers NPF k-steps ahead and feeds them to the MFMAs: the waves of a panel
//             share only the A panel, so the k-loop has no LDS writes and no barriers, and waves
//             drift freely (one's stores overlap another's MFMAs).
// diagnostics (VAP_RP_STAMPS=1): wave 0 of workgroups 0, 64, .., 448 records s_memtime at
// [0] start, [1] panel in LDS, [2 + q] start of k-step q (q < 24), [26 + nt] after N tile nt's
// stores were issued, [29] all stores done
__device__ unsigned long long g_rp_stamps[8][32];

template <int AMODE, int EPI, bool WD, bool ST = false>
__global__ __launch_bounds__(256, 2) void rowpanel_kernel(RowPanelArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[WD ? OFF_W : LDS_BYTES];
  unsigned char* P = smem;
  unsigned char* Wt = smem + OFF_W;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;  // wave w: columns w*64..+63 of the N tile
  const int nsteps = (g.N / BN) * KSTEPS;
  const int m0 = blockIdx.x * BM;
  const bf16* __restrict__ W = (const bf16*)g.W;
  const int samp = (ST && (blockIdx.x & 63) == 0 && blockIdx.x < 512 && tid == 0) ? (int)(blockIdx.x >> 6) : -1;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (samp >= 0 && k < 32) g_rp_stamps[samp][k] = t;
    }
  };
  stamp(0);
  // element offsets of row m in A and in C / add (contiguous rows, or a time chunk of each sequence)
  auto aoff = [&](int m) -> int64_t {
    if (g.rows_per_seq == 0) return (int64_t)m * g.lda;
    const int sq = m / g.rows_per_seq;
    return (int64_t)sq * g.a_seq + (int64_t)(m - sq * g.rows_per_seq) * g.lda;
  };
  auto coff = [&](int m) -> int64_t {
    if (g.rows_per_seq == 0) return (int64_t)m * g.ldc;
    const int sq = m / g.rows_per_seq;
    return (int64_t)sq * g.c_seq + (int64_t)(m - sq * g.rows_per_seq) * g.ldc;
  };

  // W staging: 1024 chunks per k-step, 4 per thread.  NPF register sets: the load for k-step
  // q + NPF is issued at step q, so an L2 round trip is hidden behind NPF steps of MFMAs.
  chunk16 rb[NPF][4];
  auto gload = [&](int q, chunk16* r) {
    const int nt = q / KSTEPS, k0 = (q % KSTEPS) * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * 256, row = id >> 2, c = id & 3;
      r[i] = g.w_packed ? *(const chunk16*)(W + ((int64_t)q * 1024 + id) * 8)
                        : *(const chunk16*)(W + (int64_t)(nt * BN + row) * KP + k0 + c * 8);
    }
  };
  auto lstore = [&](int buf, const chunk16* r) {
    unsigned char* base = Wt + buf * BN * WROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * 256;
      // packed chunk id = (16-row group, MFMA lane): row group*16 + lane%16, k chunk lane/16
      const int row = g.w_packed ? (id >> 6) * 16 + (id & 15) : id >> 2;
      const int c = g.w_packed ? (id >> 4) & 3 : id & 3;
      *(chunk16*)(base + row * WROWB + wswz(row, c) * 16) = r[i];
    }
  };
  // direct: wave w's fragment i of k-step q = W rows nt*256 + w*64 + i*16 + lane%16, 16 B at
  // k0 + (lane/16)*8 -- exactly the MFMA A-operand layout (operands are swapped)
  auto wload = [&](int q, chunk16* r) {
    const int nt = q / KSTEPS, k0 = (q % KSTEPS) * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = nt * BN + w * 64 + i * 16 + (lane & 15);
      r[i] = g.w_packed ? *(const chunk16*)(W + (((int64_t)q * 16 + w * 4 + i) * 64 + lane) * 8)
                        : *(const chunk16*)(W + (int64_t)row * KP + k0 + (lane >> 4) * 8);
    }
  };
  // (direct mode issues its W prefetch after the panel loads, so waiting for the panel does not
  // wait for W: vmcnt counts in issue order)
  auto prefetch_w = [&]() {
#pragma unroll
    for (int p = 0; p < NPF; ++p) {
      if constexpr (WD) wload(p, rb[p]);
      else gload(p, rb[p]);
    }
  };
  if constexpr (!WD) prefetch_w();

  // ------------------------------------------------------------ A panel -> LDS (bf16)
  if constexpr (AMODE == 0) {  // bf16 rows: 64 x 512 B = 2048 chunks, 8 per thread
    chunk16 t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int id = tid + i * 256, row = id >> 5, c = id & 31;
      const int m = m0 + row;
      // unconditional load of a clamped row + select: a load under a branch gets its own vmcnt(0)
      t[i] = *(const chunk16*)((const bf16*)g.A + aoff(m < g.M ? m : g.M - 1) + c * 8);
    }
    if constexpr (WD) prefetch_w();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int id = tid + i * 256, row = id >> 5, c = id & 31;
      const chunk16 v = m0 + row < g.M ? t[i] : chunk16{0, 0, 0, 0};
      *(chunk16*)(P + row * PROWB + pswz(row, c) * 16) = v;
    }
  } else {
    // fp32 rows (+ LayerNorm).  Wave w owns rows w*16 .. w*16+15 as 4 sets of 4; in one load
    // instruction each 16-lane group reads 256 contiguous bytes of its row (2 full lines), so the
    // panel streams at line granularity.  Lane (r4 = lane>>4, cc = lane&15) holds floats
    // jj*64 + cc*4 .. +3 (jj = 0..3) of row w*16 + set*4 + r4; row statistics reduce over the
    // 16-lane group.
    const int r4 = lane >> 4, cc = lane & 15;
    f32x4 v[4][4];
#pragma unroll
    for (int set = 0; set < 4; ++set) {
      const int m = m0 + w * 16 + set * 4 + r4;
      const float* src = (const float*)g.A + aoff(m < g.M ? m : g.M - 1) + cc * 4;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const f32x4 t = *(const f32x4*)(src + jj * 64);
        v[set][jj] = m < g.M ? t : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if constexpr (WD) prefetch_w();
    if constexpr (AMODE == 1) {
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
        const float mean = sum * (1.0f / KP);
        float ss = 0.f;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          v[set][jj] -= mean;
          ss += v[set][jj][0] * v[set][jj][0] + v[set][jj][1] * v[set][jj][1] + v[set][jj][2] * v[set][jj][2] +
                v[set][jj][3] * v[set][jj][3];
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) ss += __shfl_xor(ss, o, 64);
        const float rstd = rsqrtf(ss * (1.0f / KP) + g.eps);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[set][jj] = v[set][jj] * rstd * ga[jj] + be[jj];
      }
    }
#pragma unroll
    for (int set = 0; set < 4; ++set) {
      const int row = w * 16 + set * 4 + r4;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {  // 8 bytes = half of 16-byte chunk jj*8 + cc/2
        const bf16x4 b = {(bf16)v[set][jj][0], (bf16)v[set][jj][1], (bf16)v[set][jj][2], (bf16)v[set][jj][3]};
        *(bf16x4*)(P + row * PROWB + pswz(row, jj * 8 + (cc >> 1)) * 16 + (cc & 1) * 8) = b;
      }
    }
  }
  if constexpr (!WD) lstore(0, rb[0]);
  __syncthreads();
  stamp(1);

  // ------------------------------------------------------------ N tiles x k-steps
  f32x4 acc[4][4];  // [n tile 16][m tile 16] of C^T
  f32x4 radd[4][4];  // EPI 2 (WD): the tile's residual, loaded when its k-loop starts
  // WD epilogue: byte offsets of this lane's 4 output rows from the panel's first row (rows >= M:
  // out of range), buffer resources based there (a panel spans < 2 GiB of C)
  constexpr uint32_t ESZ = EPI == 2 ? 4 : 2;
  uint32_t crow[4];
  const int64_t cbase = coff(m0);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + j * 16 + (lane & 15);
    crow[j] = m < g.M ? (uint32_t)((coff(m) - cbase) * ESZ) : 0x80000000u;
  }
  const __amdgpu_buffer_rsrc_t rsrc_c = make_rsrc((const char*)g.C + cbase * ESZ, 0x7FFFFFF0u);
  const __amdgpu_buffer_rsrc_t rsrc_add =
      make_rsrc(EPI == 2 ? (const char*)g.add + cbase * ESZ : (const char*)g.C, 0x7FFFFFF0u);
  // nsteps is a multiple of KSTEPS (8), hence of NPF: unrolling by NPF makes every register-set
  // index static.
  for (int q0 = 0; q0 < nsteps; q0 += NPF) {
#pragma unroll
    for (int p = 0; p < NPF; ++p) {
      const int q = q0 + p;
      const int kq = q % KSTEPS;
      if (q < 24) stamp(2 + q);
      if (kq == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (WD && EPI == 2) {
          const int nt = q / KSTEPS;
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              radd[i][j] = __builtin_bit_cast(
                  f32x4, buf_load16(rsrc_add, crow[j] + (uint32_t)(nt * BN + w * 64 + i * 16 + (lane >> 4) * 4) * 4u, 0));
        }
      }
      chunk16 wf[4], af[4];
      if constexpr (WD) {
#pragma unroll
        for (int i = 0; i < 4; ++i) wf[i] = rb[p][i];
      } else {
        const unsigned char* wb = Wt + (q & 1) * BN * WROWB;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = w * 64 + i * 16 + (lane & 15);
          wf[i] = *(const chunk16*)(wb + row * WROWB + wswz(row, lane >> 4) * 16);
        }
      }
      const int ca = kq * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = j * 16 + (lane & 15);
        af[j] = *(const chunk16*)(P + row * PROWB + pswz(row, ca) * 16);
      }
      if constexpr (!WD) {
        if (q + NPF < nsteps) gload(q + NPF, rb[p]);  // set p held step q: stored at step q-1
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_chunk<bf16>(wf[i], af[j], acc[i][j]);
      if constexpr (WD) {
        // unconditional (the last NPF steps reload the final k-step): a conditional load makes the
        // compiler's vmcnt bookkeeping forget the younger loads and drain the whole prefetch
        wload(q + NPF < nsteps ? q + NPF : nsteps - 1, rb[p]);
      } else {
        if (q + 1 < nsteps) lstore((q + 1) & 1, rb[(p + 1) % NPF]);
      }
      if (kq == KSTEPS - 1) {
        // epilogue of N tile nt: lane owns C[m][n .. n+3]
        const int nt = q / KSTEPS;
        if constexpr (WD) {
          // branch-free: rows >= M carry an out-of-range offset and their stores are dropped
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uint32_t n = nt * BN + w * 64 + i * 16 + (lane >> 4) * 4;
              f32x4 v = acc[i][j];
              if constexpr (EPI == 1) {
const f32x2 lo = gelu_fast2((f32x2){v[0], v[1]}), hi = gelu_fast2((f32x2){v[2], v[3]});
                v = f32x4{lo[0], lo[1], hi[0], hi[1]};
              }
              if constexpr (EPI == 2) {
                v += radd[i][j];
                buf_store16_wt(rsrc_c, crow[j] + n * 4u, __builtin_bit_cast(u32x4, v));
              } else {
                buf_store8(rsrc_c, crow[j] + n * 2u, pack_bf16x4(v[0], v[1], v[2], v[3]));
              }
            }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int m = m0 + j * 16 + (lane & 15);
            if (m >= g.M) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int n = nt * BN + w * 64 + i * 16 + (lane >> 4) * 4;
              f32x4 v = acc[i][j];
              if constexpr (EPI == 1) {
const f32x2 lo = gelu_fast2((f32x2){v[0], v[1]}), hi = gelu_fast2((f32x2){v[2], v[3]});
                v = f32x4{lo[0], lo[1], hi[0], hi[1]};
              }
              const int64_t co = coff(m) + n;
              if constexpr (EPI == 2) {
                v += *(const f32x4*)((const float*)g.add + co);
                *(f32x4*)((float*)g.C + co) = v;
              } else {
                store4((bf16*)g.C + co, v[0], v[1], v[2], v[3]);
              }
            }
          }
        }
        if (q / KSTEPS < 3) stamp(26 + q / KSTEPS);
      }
      if constexpr (!WD) __syncthreads();
    }
  }
  if constexpr (ST) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(29);
  }
}

}  // namespace

hipError_t launch_rowpanel(const RowPanelArgs& g, int amode, int epi, hipStream_t st) {
  if (g.M <= 0 || g.N % BN != 0 || g.K != KP || g.rows_per_seq < 0) return hipErrorInvalidValue;
  // the epilogue's buffer offsets reach 2 GiB from a panel's first output row
  const int64_t span = g.rows_per_seq ? (BM / g.rows_per_seq + 2) * g.c_seq + (int64_t)BM * g.ldc : (int64_t)BM * g.ldc;
  if (span * (epi == 2 ? 4 : 2) >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
  const dim3 grid((g.M + BM - 1) / BM);
  static const bool v1 = getenv("VAP_RP_V1") != nullptr;
  static const bool stamps = getenv("VAP_RP_STAMPS") != nullptr;
  if (stamps && amode == 1 && epi <= 1) {  // diagnostics build of the LayerNorm'd projections
    if (v1 && epi == 0) hipLaunchKernelGGL((rowpanel_kernel<1, 0, false, true>), grid, dim3(256), 0, st, g);
    else if (v1) hipLaunchKernelGGL((rowpanel_kernel<1, 1, false, true>), grid, dim3(256), 0, st, g);
    else if (epi == 0) hipLaunchKernelGGL((rowpanel_kernel<1, 0, true, true>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((rowpanel_kernel<1, 1, true, true>), grid, dim3(256), 0, st, g);
    return hipGetLastError();
  }
#define RP_LAUNCH(A, E)                                                                      \
  do {                                                                                       \
    if (v1) hipLaunchKernelGGL((rowpanel_kernel<A, E, false>), grid, dim3(256), 0, st, g);   \
    else hipLaunchKernelGGL((rowpanel_kernel<A, E, true>), grid, dim3(256), 0, st, g);       \
  } while (0)
  if (amode == 0 && epi == 0) RP_LAUNCH(0, 0);
  else if (amode == 0 && epi == 2) RP_LAUNCH(0, 2);
  else if (amode == 1 && epi == 0) RP_LAUNCH(1, 0);
  else if (amode == 1 && epi == 1) RP_LAUNCH(1, 1);
  else if (amode == 2 && epi == 0) RP_LAUNCH(2, 0);
  else return hipErrorInvalidValue;
#undef RP_LAUNCH
  return hipGetLastError();
}

// diagnostics: copy the row-panel stamps (8 sampled workgroups x 32) to host memory
hipError_t read_rowpanel_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rp_stamps), sizeof(g_rp_stamps), 0, hipMemcpyDeviceToHost);
}
