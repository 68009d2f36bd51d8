// MFMA GEMM with implicit-convolution A addressing and fused row epilogues.
//
//   C[m, n] = epi( sum_k A[m, k] * W[n, k] )          (W = weight [N][K], K-contiguous)
//   A row m = (seq s, frame t):  A + s*a_seq_stride + t*lda        (rows may OVERLAP: lda < K)
//
// Overlapping rows turn a strided Conv1d over a time-major [pos][ch] activation into a plain
// GEMM with no im2col buffer:  conv k=8,s=4 (CPC conv1): lda = 4*256, K = 8*256;
// conv k=4,s=2 (conv2..4): lda = 512, K = 1024; causal k=5,s=2 downsample: lda = 512, K = 1280
// (reference: vap/encoder_components.py:83-92, 428-499).  Zero padding lives in explicit pad rows of
// the activation buffers, so the loader never branches on the conv border.
//
// Epilogue (one code path, uniform runtime switches):
//   v = acc + bias;  v = norm(v) [ChannelNorm: unbiased var (encoder_components.py:62-70) |
//   LayerNorm: biased var (nn.LayerNorm)] * gamma + beta;  v = act(v) [relu | gelu(erf)];
//   v += add (fp32 residual / combinator partial);  store as TOut.
// Row norms need the whole 256-wide row in one workgroup: BN = 256.
//
// Tile 128 x 256, 8 waves (2 along M x 4 along N, 64x64 per wave = 4x4 MFMA 16x16 tiles),
// K staged 128 bytes per row per step (64 bf16 / 32 f32) through a double-buffered, XOR-swizzled
// LDS image (chunk ^= (row>>1)&7 : conflict-free ds_read_b128 for 16 consecutive rows).
//
// gemm3_kernel (the fp32 parity mode's GEMMs, GemmArgs.split): fp32 A and W at ~fp32 accuracy on the
// bf16 matrix cores.  Every fp32 operand x is split as x = hi + lo with hi = bf16(x), lo = bf16(x - hi)
// (x - hi - lo ~ 2^-17 |x|), and each product as hi_a hi_w + hi_a lo_w + lo_a hi_w (the lo lo term is
// ~2^-18 of it), three v_mfma_f32_16x16x32_bf16 with fp32 accumulation: 3 x 16 cycles per 16x16x32
// tile-step instead of 8 x 32 for v_mfma_f32_16x16x4_f32 (5.3x the matrix rate).  W arrives pre-split
// (launch_split_bf16); A is split once per workgroup while it is staged to LDS.
#include <cstdlib>
#include <type_traits>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

constexpr int BM = 128, BN = 256, ROWB = 128;  // bytes per staged row
constexpr int BUF = (BM + BN) * ROWB;          // 48 KiB per stage

VAP_DEV int swz(int row, int c) { return c ^ ((row >> 1) & 7); }

// fused epilogue of a 128 x 256 tile (wave (wm, wn) holds acc[i][j] = 16x16 tile (rows wm*64 + 16i,
// cols wn*64 + 16j)): bias, row norm, activation, fp32 addend, store.  smem: >= BM*4 floats, free.
template <typename TOut>
VAP_DEV void gemm_epilogue(const GemmArgs& g, f32x4 (&acc)[4][4], unsigned char* smem, int m0, int n0, int wm, int wn,
                           int lane, int M) {
  const int colb = n0 + wn * 64 + (lane & 15);
  if (g.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float b = g.bias[colb + j * 16];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] += b;
    }
  }
  if (g.norm) {
    float* red = (float*)smem;  // [BM][4]
    float mean[4][4], rstd[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = acc[i][0][r] + acc[i][1][r] + acc[i][2][r] + acc[i][3][r];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        const int rl = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if ((lane & 15) == 0) red[rl * 4 + wn] = s;
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const f32x4 p = *(const f32x4*)(red + rl * 4);
        mean[i][r] = (p[0] + p[1] + p[2] + p[3]) * (1.0f / BN);
      }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = acc[i][j][r] - mean[i][r];
          s += d * d;
        }
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        const int rl = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        if ((lane & 15) == 0) red[rl * 4 + wn] = s;
      }
    __syncthreads();
    const float inv_n = g.norm == 1 ? 1.0f / (BN - 1) : 1.0f / BN;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const f32x4 p = *(const f32x4*)(red + rl * 4);
        const float var = (p[0] + p[1] + p[2] + p[3]) * inv_n;
        rstd[i][r] = rsqrtf(var + g.eps);
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float ga = g.gamma[colb + j * 16], be = g.beta[colb + j * 16];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = (acc[i][j][r] - mean[i][r]) * rstd[i][r] * ga + be;
    }
  }
  if (g.act == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = fmaxf(acc[i][j][r], 0.f);
  } else if (g.act == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = gelu_erf(acc[i][j][r]);
  }
  // store: each 16-row slab of the wave's 64 x 64 block is transposed through a wave-private LDS area
  // ([16][68] floats; rows padded so the scalar writes of two 16-lane row groups hit distinct banks), so
  // every lane then holds 4 consecutive columns of one row: 16-B loads of the addend and 16-B stores, 256
  // contiguous bytes per 16 lanes (the accumulator layout gave one 4-B element per lane, 64-B segments)
  TOut* __restrict__ C = (TOut*)g.C;
  float* tp = (float*)(smem + 4096) + (wm * 4 + wn) * (16 * 68);
  const int cl = (lane & 15) * 4;  // the lane's 4 columns of the wave's 64 after the transpose
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) tp[((lane >> 4) * 4 + r) * 68 + j * 16 + (lane & 15)] = acc[i][j][r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int rr = p * 4 + (lane >> 4);  // row of the slab
      f32x4 v = *(const f32x4*)(tp + rr * 68 + cl);
      const int m = m0 + wm * 64 + i * 16 + rr;
      if (m < M) {
        const int s = m / g.M_per_seq, t = m - s * g.M_per_seq;
        const int col = n0 + wn * 64 + cl;
        if (g.add) v += *(const f32x4*)(g.add + (int64_t)s * g.add_seq_stride + (int64_t)t * g.ld_add + col);
        store4(C + (int64_t)s * g.c_seq_stride + (int64_t)t * g.ldc + col, v[0], v[1], v[2], v[3]);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the slab is read before the next one overwrites it
  }
}

template <typename T, typename TOut>
__global__ __launch_bounds__(512) void gemm_kernel(GemmArgs g) {
  constexpr int CE = 16 / sizeof(T);  // elements per 16-B chunk
  constexpr int BK = 8 * CE;          // k per stage
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int M = g.M_per_seq * g.n_seq;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const T* __restrict__ A = (const T*)g.A;
  const T* __restrict__ W = (const T*)g.W;

  // ---- staging assignment: A 1024 chunks (2 / thread), B 2048 chunks (4 / thread)
  const T* aptr[2];
  bool aval[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + i * 512, row = id >> 3, c = id & 7;
    const int m = m0 + row;
    aval[i] = m < M;
    const int mm = aval[i] ? m : 0;
    const int s = mm / g.M_per_seq, t = mm - s * g.M_per_seq;
    aptr[i] = A + (int64_t)s * g.a_seq_stride + (int64_t)t * g.lda + c * CE;
  }
  const T* bptr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + i * 512, row = id >> 3, c = id & 7;
    bptr[i] = W + (int64_t)(n0 + row) * g.K + c * CE;
  }
  chunk16 ra[2], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = aval[i] ? *(const chunk16*)(aptr[i] + k0) : chunk16{0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; ++i) rb[i] = *(const chunk16*)(bptr[i] + k0);
  };
  auto lstore = [&](int buf) {
    unsigned char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + i * 512, row = id >> 3, c = id & 7;
      *(chunk16*)(base + row * ROWB + swz(row, c) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * 512, row = id >> 3, c = id & 7;
      *(chunk16*)(base + BM * ROWB + row * ROWB + swz(row, c) * 16) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    const unsigned char* abase = smem + cur * BUF;
    const unsigned char* bbase = abase + BM * ROWB;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      chunk16 af[4], bfr[4];
      const int c = sub * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + (lane & 15);
        af[i] = *(const chunk16*)(abase + row * ROWB + swz(row, c) * 16);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + j * 16 + (lane & 15);
        bfr[j] = *(const chunk16*)(bbase + row * ROWB + swz(row, c) * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_chunk<T>(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  gemm_epilogue<TOut>(g, acc, smem, m0, n0, wm, wn, lane, M);
}


// fp32 A x split W on the bf16 matrix cores (see the header): C = epi(A . W^T) at ~fp32 accuracy.
// Stage = 32 k.  Every staged row is 128 B = [hi of the 32 k | lo of the 32 k] (chunks 0-3 hi, 4-7 lo),
// swizzled as the bf16 kernel's rows (chunk ^= (row>>1)&7): a wave's hi and lo fragment reads are
// exactly that kernel's two sub-steps, conflict-free.  A stage is 48 KiB (A 16 + W 32), double-buffered
// as in gemm_kernel (one barrier per stage; the next stage is loaded into registers during the MFMAs).
// W arrives pre-split in the same row format ([N][K/32][64] bf16, launch_split_bf16 with K); thread t
// stages 2 A chunks (4 floats: row id >> 3, k 4 (id & 7), split into 8-B hi / lo halves) and 4 W chunks.
__global__ __launch_bounds__(512) void gemm3_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int M = g.M_per_seq * g.n_seq;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const float* A = (const float*)g.A;
  const bf16* W = (const bf16*)g.W;

  // loads through buffer resources: one 32-bit lane offset per chunk, the stage as a scalar offset; A rows
  // past M read as zero (offset outside the resource), no branches (a conditional load made the compiler
  // drain every load in flight); A's resource starts at the tile's first sequence (the host checks that
  // the tile's rows lie within the 2 GiB a buffer offset reaches)
  const int sq0 = m0 / g.M_per_seq;
  const __amdgpu_buffer_rsrc_t rA = make_rsrc(A + (int64_t)sq0 * g.a_seq_stride, 0x7FFFFFF0u);
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, 0x7FFFFFF0u);
  uint32_t aoff[2], woff[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + i * 512, row = id >> 3, c = id & 7;
    const int m = m0 + row;
    const int s = m / g.M_per_seq, t = m - s * g.M_per_seq;
    aoff[i] = m < M ? (uint32_t)((((int64_t)(s - sq0) * g.a_seq_stride + (int64_t)t * g.lda) + c * 4) * 4) : 0x80000000u;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + i * 512, row = id >> 3, c = id & 7;
    woff[i] = (uint32_t)(((int64_t)(n0 + row) * (2 * g.K) + c * 8) * 2);
  }
  // A (streamed from HBM) is prefetched three stages ahead through a ring of register sets, W (L2-resident,
  // small) one stage ahead: issued W(k+1) first, then A(k+3), so the wait for W(k+1) leaves A(k+3) in flight
  chunk16 ra[3][2], rb[4];
  auto gloadA = [&](int kt, chunk16 (&r)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = buf_load16(rA, aoff[i], (uint32_t)kt * 128u);
  };
  auto gloadW = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) rb[i] = buf_load16(rW, woff[i], (uint32_t)kt * 128u);
  };
  auto lstore = [&](int buf, const chunk16 (&ra)[2]) {
    unsigned char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + i * 512, row = id >> 3, c = id & 7;  // floats 4c .. 4c+3 -> bf16 bytes 8c .. 8c+7 of a half
      const f32x4 v = __builtin_bit_cast(f32x4, ra[i]);
      const bf16x4 hi = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      const bf16x4 lo = {(bf16)(v[0] - (float)hi[0]), (bf16)(v[1] - (float)hi[1]), (bf16)(v[2] - (float)hi[2]),
                         (bf16)(v[3] - (float)hi[3])};
      *(bf16x4*)(base + row * ROWB + swz(row, c >> 1) * 16 + (c & 1) * 8) = hi;
      *(bf16x4*)(base + row * ROWB + swz(row, 4 + (c >> 1)) * 16 + (c & 1) * 8) = lo;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + i * 512, row = id >> 3, c = id & 7;
      *(chunk16*)(base + BM * ROWB + row * ROWB + swz(row, c) * 16) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / 32;
  gloadW(0);
  gloadA(0, ra[0]);
  if (nk > 1) gloadA(1, ra[1]);
  if (nk > 2) gloadA(2, ra[2]);
  lstore(0, ra[0]);
  __syncthreads();
  auto stage = [&](int kt, auto slot) {
    constexpr int S0 = decltype(slot)::value, S1 = (S0 + 1) % 3;  // ring slots of stages kt (and kt+3), kt+1
    const int cur = kt & 1;
    if (kt + 1 < nk) gloadW(kt + 1);
    if (kt + 3 < nk) gloadA(kt + 3, ra[S0]);
    const unsigned char* abase = smem + cur * BUF;
    const unsigned char* bbase = abase + BM * ROWB;
    chunk16 ah[4], al[4], bh[4], bl[4];
    const int c = lane >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + (lane & 15);
      ah[i] = *(const chunk16*)(abase + row * ROWB + swz(row, c) * 16);
      al[i] = *(const chunk16*)(abase + row * ROWB + swz(row, 4 + c) * 16);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + j * 16 + (lane & 15);
      bh[j] = *(const chunk16*)(bbase + row * ROWB + swz(row, c) * 16);
      bl[j] = *(const chunk16*)(bbase + row * ROWB + swz(row, 4 + c) * 16);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = mfma_chunk<bf16>(ah[i], bl[j], acc[i][j]);
        acc[i][j] = mfma_chunk<bf16>(al[i], bh[j], acc[i][j]);
        acc[i][j] = mfma_chunk<bf16>(ah[i], bh[j], acc[i][j]);
      }
    if (kt + 1 < nk) lstore(cur ^ 1, ra[S1]);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 3) {
    stage(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nk) stage(kt + 1, std::integral_constant<int, 1>{});
    if (kt + 2 < nk) stage(kt + 2, std::integral_constant<int, 2>{});
  }
  gemm_epilogue<float>(g, acc, smem, m0, n0, wm, wn, lane, M);
}

// fp32 W [N][K] -> the split row format of gemm3_kernel: out[n][kb][0..31] = hi, [32..63] = lo of
// W[n][32kb .. 32kb + 31] (hi = bf16(x), lo = bf16(x - hi): x = hi + lo + O(2^-17 |x|))
__global__ void split_bf16_kernel(const float* __restrict__ in, bf16* __restrict__ out, int64_t n, int K) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = in[i];
    const bf16 hi = (bf16)x;
    const int64_t row = i / K;
    const int k = (int)(i - row * K);
    bf16* o = out + row * 2 * K + (k >> 5) * 64 + (k & 31);
    o[0] = hi;
    o[32] = (bf16)(x - (float)hi);
  }
}

}  // namespace

template <typename T, typename TOut>
hipError_t launch_gemm(const GemmArgs& g, hipStream_t st) {
  const int M = g.M_per_seq * g.n_seq;
  constexpr int BK = 8 * (16 / sizeof(T));
  if (g.K % BK != 0 || g.N % BN != 0 || M <= 0) return hipErrorInvalidValue;
  if (g.norm && g.N != BN) return hipErrorInvalidValue;
  if constexpr (sizeof(T) == 2) {
    const bool aligned = !(g.lda % 8 || g.a_seq_stride % 8 || g.ldc % 4 || g.c_seq_stride % 4 ||
                           (g.add && (g.ld_add % 4 || g.add_seq_stride % 4)));
    // The kernel choice must not depend on M: a clip's outputs are then bit-identical whatever
    // batch (or shard of a batch) it runs in -- the 128-row kernel accumulates in another order.
    if (aligned && !g.small_tiles) return launch_gemm2<TOut>(g, st);
  }
  // the epilogue's 16-B (fp32) / 8-B (bf16) row stores and addend loads need aligned rows
  const uintptr_t al = 4 * sizeof(TOut) - 1;
  if (g.ldc % 4 || g.c_seq_stride % 4 || ((uintptr_t)g.C & al) ||
      (g.add && (g.ld_add % 4 || g.add_seq_stride % 4 || ((uintptr_t)g.add & 15))))
    return hipErrorInvalidValue;
  dim3 grid((M + BM - 1) / BM, g.N / BN);
  if constexpr (sizeof(T) == 4 && sizeof(TOut) == 4) {
    if (g.split) {  // fp32 operands through the split-bf16 kernel (W: launch_split_bf16's row format)
      if (g.K % 32 != 0) return hipErrorInvalidValue;
      // a tile's A rows (at most BM / M_per_seq + 2 sequences) and the split W lie within a buffer offset's 2 GiB
      if ((((int64_t)BM / g.M_per_seq + 2) * g.a_seq_stride + (int64_t)BM * g.lda + g.K) * 4 >= 0x7FFFFFF0LL ||
          (int64_t)g.N * g.K * 4 >= 0x7FFFFFF0LL)
        return hipErrorInvalidValue;
      hipLaunchKernelGGL(gemm3_kernel, grid, dim3(512), 0, st, g);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_kernel<T, TOut>), grid, dim3(512), 0, st, g);
  return hipGetLastError();
}

hipError_t launch_split_bf16(const float* in, bf16* out, int64_t n, int K, hipStream_t st) {
  if (n <= 0 || K <= 0 || K % 32 || n % K) return hipErrorInvalidValue;
  hipLaunchKernelGGL(split_bf16_kernel, dim3(256), dim3(256), 0, st, in, out, n, K);
  return hipGetLastError();
}

template hipError_t launch_gemm<bf16, bf16>(const GemmArgs&, hipStream_t);
template hipError_t launch_gemm<bf16, float>(const GemmArgs&, hipStream_t);
template hipError_t launch_gemm<float, float>(const GemmArgs&, hipStream_t);
