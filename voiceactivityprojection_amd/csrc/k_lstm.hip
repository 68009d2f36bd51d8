// LSTM recurrence of CPCAR (vap/encoder_components.py:107-159 -> nn.LSTM, batch_first, zero
// initial state, gates i,f,g,o).  The input projection x W_ih^T + b_ih + b_hh for all frames is
// a plain GEMM done beforehand (gx, fp32); this kernel runs the serial part:
//   z_t = gx_t + h_{t-1} W_hh^T ;  c_t = s(f) c_{t-1} + s(i) tanh(g) ;  h_t = s(o) tanh(c_t)
//
// One workgroup = 16 sequences (the MFMA N dimension), 4 waves; wave w owns hidden units
// [64w, 64w+64) and therefore gate rows {g*256 + 64w + u}: the four gates of a unit land in the
// same lane/register of four accumulator tiles, so the cell update is purely lane-local.
// h_{t-1} is exchanged through a padded LDS image (one barrier per step); W_hh is pre-packed in
// MFMA-fragment order so every wave-load is one contiguous KiB.
#include "vap_common.h"
#include "vap_kernels.h"

namespace {

constexpr int HD = 256, G4 = 1024, NS = 16;

template <typename T>
struct LstmGeom {
  static constexpr int CE = 16 / sizeof(T);     // k per lane per chunk
  static constexpr int KG = HD / (4 * CE);      // k-groups per row (8 bf16 / 16 f32)
  static constexpr int HROW = HD * sizeof(T) + 16;  // padded LDS row bytes
};

template <typename T>
__global__ __launch_bounds__(256) void lstm_kernel(const float* __restrict__ gx, int S, int Tn,
                                                  const chunk16* __restrict__ whh, T* __restrict__ out,
                                                  int64_t out_seq_stride) {
  using Gm = LstmGeom<T>;
  __shared__ __attribute__((aligned(16))) unsigned char hbuf[2][NS * Gm::HROW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int seq = blockIdx.x * NS + (lane & 15);
  const bool valid = seq < S;
  for (int i = tid; i < 2 * NS * Gm::HROW / 4; i += 256) ((unsigned*)hbuf)[i] = 0u;
  float c[4][4];
#pragma unroll
  for (int ut = 0; ut < 4; ++ut)
#pragma unroll
    for (int r = 0; r < 4; ++r) c[ut][r] = 0.f;
  __syncthreads();

  const float* gxs = gx + (int64_t)(valid ? seq : 0) * Tn * G4;
  const chunk16* wbase = whh + (int64_t)w * 16 * Gm::KG * 64 + lane;
  for (int t = 0; t < Tn; ++t) {
    const unsigned char* hcur = hbuf[t & 1];
    unsigned char* hnext = hbuf[(t + 1) & 1];
    f32x4 acc[4][4];
    const float* gxt = gxs + (int64_t)t * G4 + 64 * w + (lane >> 4) * 4;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int ut = 0; ut < 4; ++ut)
        acc[g][ut] = valid ? *(const f32x4*)(gxt + g * HD + ut * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int kg = 0; kg < Gm::KG; ++kg) {
      const chunk16 hb = *(const chunk16*)(hcur + (lane & 15) * Gm::HROW + (kg * 4 + (lane >> 4)) * 16);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int ut = 0; ut < 4; ++ut) {
          const chunk16 a = wbase[((g * 4 + ut) * Gm::KG + kg) * 64];
          acc[g][ut] = mfma_chunk<T>(a, hb, acc[g][ut]);
        }
    }
    // cell update: unit u = 64w + 16ut + (lane>>4)*4 + r, sequence lane&15
#pragma unroll
    for (int ut = 0; ut < 4; ++ut) {
      float h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ig = 1.0f / (1.0f + expf(-acc[0][ut][r]));
        const float fg = 1.0f / (1.0f + expf(-acc[1][ut][r]));
        const float gg = tanhf(acc[2][ut][r]);
        const float og = 1.0f / (1.0f + expf(-acc[3][ut][r]));
        c[ut][r] = fg * c[ut][r] + ig * gg;
        h[r] = og * tanhf(c[ut][r]);
      }
      const int u = 64 * w + 16 * ut + (lane >> 4) * 4;
      store4((T*)(hnext + (lane & 15) * Gm::HROW) + u, h[0], h[1], h[2], h[3]);
      if (valid) store4(out + (int64_t)seq * out_seq_stride + (int64_t)t * HD + u, h[0], h[1], h[2], h[3]);
    }
    __syncthreads();
  }
}

// Wp[((w*16 + g*4 + ut)*KG + kg)*64 + l][e] = W[g*256 + 64w + 16ut + (l&15)][kg*4*CE + (l>>4)*CE + e]
template <typename T>
__global__ void pack_whh_kernel(const float* __restrict__ whh, T* __restrict__ out) {
  using Gm = LstmGeom<T>;
  constexpr int CE = Gm::CE;
  const int64_t n = (int64_t)G4 * HD;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(i % CE);
    int64_t q = i / CE;
    const int l = (int)(q % 64);
    q /= 64;
    const int kg = (int)(q % Gm::KG);
    q /= Gm::KG;
    const int tile = (int)(q % 16), w = (int)(q / 16);
    const int g = tile / 4, ut = tile % 4;
    const int row = g * HD + 64 * w + 16 * ut + (l & 15);
    const int k = kg * 4 * CE + (l >> 4) * CE + e;
    out[i] = from_f32<T>(whh[(int64_t)row * HD + k]);
  }
}

}  // namespace

template <typename T>
hipError_t launch_lstm(const float* gx, int S, int Tn, const T* whh_packed, T* out, int64_t out_seq_stride,
                       hipStream_t st) {
  if (S <= 0 || Tn <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL((lstm_kernel<T>), dim3((S + NS - 1) / NS), dim3(256), 0, st, gx, S, Tn,
                     (const chunk16*)whh_packed, out, out_seq_stride);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pack_whh(const float* whh, T* packed, hipStream_t st) {
  hipLaunchKernelGGL((pack_whh_kernel<T>), dim3(256), dim3(256), 0, st, whh, packed);
  return hipGetLastError();
}

template hipError_t launch_lstm<float>(const float*, int, int, const float*, float*, int64_t, hipStream_t);
template hipError_t launch_lstm<bf16>(const float*, int, int, const bf16*, bf16*, int64_t, hipStream_t);
template hipError_t launch_pack_whh<float>(const float*, float*, hipStream_t);
template hipError_t launch_pack_whh<bf16>(const float*, bf16*, hipStream_t);
