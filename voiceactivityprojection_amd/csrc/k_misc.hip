// Memory-bound kernels of the VAP path: conv0 + ChannelNorm + ReLU, LayerNorm, the
// va_classifier head, the probs() epilogue and label extraction + cross entropy.
#include <algorithm>

#include "vap_common.h"
#include "vap_kernels.h"

namespace {

// ------------------------------------------------------------------------------------------
// conv0 (1 -> 256, k=10, s=5, p=3) -> ChannelNorm (unbiased var over 256 ch, eps 1e-5) -> ReLU
// reference: vap/encoder_components.py:83-84 (conv0/batchNorm0), :62-70 (ChannelNorm), :99.
// (fp32 parity mode; the bf16 mode fuses conv0 into conv1, k_conv01.hip.)  Store-bound: the
// output is 1 KiB per position (fp32), 131 MB per 20 s stereo clip.  Block = 64 positions of one
// sequence (seq = 2*clip + channel); lane l owns channels 4l .. 4l+3 (its 40 weights in registers),
// wave w positions 16w .. 16w+15: every output row leaves as ONE 1 KiB store instruction (16 B per
// lane, fully coalesced), the row statistics by wave reductions.  The 326 samples of the block are
// staged in LDS and read as broadcasts.  Output time-major [seq][2 + L0 + 2][256] (2 pad rows each
// side = conv1's zero padding).
// ------------------------------------------------------------------------------------------
constexpr int C0 = 256, KW0 = 10, P0 = 64, NSMP = P0 * 5 + 6;

template <typename T>
__global__ __launch_bounds__(256) void conv0_kernel(const float* __restrict__ wav, int B, int64_t N, int L0,
                                                   const float* __restrict__ w0, const float* __restrict__ b0,
                                                   const float* __restrict__ gam, const float* __restrict__ bet,
                                                   T* __restrict__ out, int64_t out_seq_stride) {
  __shared__ float smp[NSMP + 2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int s = blockIdx.y;  // sequence = 2 * clip + channel (clip-major == the [B][2][N] waveform)
  const int p0 = blockIdx.x * P0;
  const float* src = wav + (int64_t)s * N;
  const int64_t i0 = (int64_t)p0 * 5 - 3;
  for (int i = tid; i < NSMP; i += 256) {
    const int64_t j = i0 + i;
    smp[i] = (j >= 0 && j < N) ? src[j] : 0.f;
  }
  float wv[4][KW0], bv[4], gv[4], be[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = 4 * lane + e;
#pragma unroll
    for (int k = 0; k < KW0; ++k) wv[e][k] = w0[c * KW0 + k];
    bv[e] = b0[c];
    gv[e] = gam[c];
    be[e] = bet[c];
  }
  __syncthreads();
#pragma unroll 2
  for (int j = 0; j < 16; ++j) {
    const int pl = w * 16 + j, pos = p0 + pl;
    if (pos >= L0) break;  // wave-uniform
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = bv[e];
#pragma unroll
      for (int k = 0; k < KW0; ++k) v = fmaf(wv[e][k], smp[pl * 5 + k], v);
      x[e] = v;
    }
    const float mean = wave_sum((x[0] + x[1]) + (x[2] + x[3])) * (1.0f / C0);
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) ss = fmaf(x[e] - mean, x[e] - mean, ss);
    const float rstd = rsqrtf(wave_sum(ss) * (1.0f / (C0 - 1)) + 1e-5f);
    float y[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = fmaxf((x[e] - mean) * rstd * gv[e] + be[e], 0.f);
    store4(out + (int64_t)s * out_seq_stride + (int64_t)(pos + 2) * C0 + 4 * lane, y[0], y[1], y[2], y[3]);
  }
}

template <typename T>
__global__ void zero_rows_kernel(T* base, int64_t seq_stride, int rows) {
  const int s = blockIdx.y;
  const int64_t n = (int64_t)rows * 256;
  T* p = base + (int64_t)s * seq_stride;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = from_f32<T>(0.f);
}

// every region's pad rows in one launch: region r = blockIdx.z, sequence = blockIdx.y
__global__ void zero_regions_kernel(ZeroRegions z) {
  const ZeroRegion& r = z.r[blockIdx.z];
  const int64_t n = r.bytes / 16;  // 16-byte words per sequence (rows x 256 x element size)
  unsigned char* p = (unsigned char*)r.base + (int64_t)blockIdx.y * r.seq_stride_bytes;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ((u32x4*)p)[i] = u32x4{0u, 0u, 0u, 0u};
}

// ------------------------------------------------------------------------------------------
// LayerNorm over 256 (nn.LayerNorm, biased var) -- one wave per row, 4 values per lane.
// Optional raw copy (cross-attention K/V source is the UN-normalised x: modules.py:265-272).
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t rows,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, T* __restrict__ out, T* __restrict__ raw) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const f32x4 v = *(const f32x4*)(x + row * 256 + lane * 4);
  if (raw) store4(raw + row * 256 + lane * 4, v[0], v[1], v[2], v[3]);
  if (!gamma) return;
  const float mean = wave_sum(v[0] + v[1] + v[2] + v[3]) * (1.0f / 256);
  const f32x4 d = v - mean;
  const float var = wave_sum(d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3]) * (1.0f / 256);
  const float rstd = rsqrtf(var + eps);
  const f32x4 g = *(const f32x4*)(gamma + lane * 4);
  const f32x4 b = *(const f32x4*)(beta + lane * 4);
  const f32x4 y = d * rstd * g + b;
  store4(out + row * 256 + lane * 4, y[0], y[1], y[2], y[3]);
}

// va_classifier (model.py:162,258-260): vad[b][t][c] = x_c[b,t] . w + bias; x rows fp32 channel-major
__global__ __launch_bounds__(256) void vad_head_kernel(const float* __restrict__ x, int B, int Tn,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      float* __restrict__ vad) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // row over (seq = 2b + c, t)
  const int64_t rows = (int64_t)2 * B * Tn;
  if (row >= rows) return;
  const f32x4 v = *(const f32x4*)(x + row * 256 + lane * 4);
  const f32x4 ww = *(const f32x4*)(w + lane * 4);
  const float d = wave_sum(v[0] * ww[0] + v[1] * ww[1] + v[2] * ww[2] + v[3] * ww[3]) + bias[0];
  if (lane == 0) {
    const int64_t s = row / Tn, t = row - s * Tn;
    vad[((s >> 1) * Tn + t) * 2 + (s & 1)] = d;
  }
}

// frame range variant (time-chunked back end): row over (seq, t in [t0, t0 + nt))
__global__ __launch_bounds__(256) void vad_head_rows_kernel(const float* __restrict__ x, int64_t x_seq, int B, int Tn,
                                                           int t0, int nt, const float* __restrict__ w,
                                                           const float* __restrict__ bias, float* __restrict__ vad) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)2 * B * nt) return;
  const int64_t s = row / nt, t = row - s * nt;
  const f32x4 v = *(const f32x4*)(x + s * x_seq + t * 256 + lane * 4);
  const f32x4 ww = *(const f32x4*)(w + lane * 4);
  const float d = wave_sum(v[0] * ww[0] + v[1] * ww[1] + v[2] * ww[2] + v[3] * ww[3]) + bias[0];
  if (lane == 0) vad[((s >> 1) * Tn + t0 + t) * 2 + (s & 1)] = d;
}

template <typename T>
__global__ __launch_bounds__(256) void convert_rows_kernel(const float* __restrict__ in, int64_t in_seq,
                                                          T* __restrict__ out, int64_t out_seq, int n_seq, int rows) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // 4 elements each
  const int64_t per_seq = (int64_t)rows * 64;
  if (i >= per_seq * n_seq) return;
  const int64_t s = i / per_seq, e = (i - s * per_seq) * 4;
  const f32x4 v = *(const f32x4*)(in + s * in_seq + e);
  store4(out + s * out_seq + e, v[0], v[1], v[2], v[3]);
}

// ------------------------------------------------------------------------------------------
// probs() epilogue (model.py:189-213): softmax, sigmoid VAD, entropy H = sum -p log2 p, and
// probs_next_speaker_aggregate (objective.py:184-204) for the now / future bin ranges:
//   abp[k, c] = popcount(bits of k in [c*nb+from, c*nb+to]);  p = probs . abp;  p /= sum_c p + 1e-5
// One 16-lane row per frame (4 frames per wave), 16 classes per lane: lane l holds classes
// 64k + 4l .. +3 (k = 0..3), so each of the four 16-B loads of a row reads 256 contiguous bytes,
// and every reduction is 4 DPP steps inside the row (a wave per frame took 6 steps per reduction
// for 4 classes per lane, and one 16-B load per lane: 45 us per bench epilogue).
// ------------------------------------------------------------------------------------------
VAP_DEV float row_sum16(float v) {  // sum over the lane's 16-lane row; every lane gets the same bits
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}
VAP_DEV float row_max16(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
// Softmax pieces of one frame's 256 logits `lg` held by a 16-lane row: e = exp(x - max), its sum.
// Shared by probs_kernel, labels_loss_kernel and probs_loss_kernel, so their outputs are bit-identical.
VAP_DEV void soft16_load(const float* __restrict__ lg, int l16, f32x4 (&e)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = *(const f32x4*)(lg + 64 * k + 4 * l16);
}
VAP_DEV void soft16_exp(f32x4 (&e)[4], float& mx, float& sum) {  // logits in e -> exp(x - max) in e
  float m = e[0][0];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) m = fmaxf(m, e[k][i]);
  mx = row_max16(m);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int i = 0; i < 4; ++i) e[k][i] = expf(e[k][i] - mx);
    s += (e[k][0] + e[k][1]) + (e[k][2] + e[k][3]);
  }
  sum = row_sum16(s);
}
VAP_DEV void soft16(const float* __restrict__ lg, int l16, f32x4 (&e)[4], float& mx, float& sum) {
  soft16_load(lg, l16, e);
  soft16_exp(e, mx, sum);
}
// probs, H, p_now / p_future of one frame from soft16's pieces (lane l16 of the frame's row);
// the row's lane 0 writes the per-frame scalars and the VAD sigmoid.
VAP_DEV void probs_frame(int64_t f, int l16, f32x4 (&e)[4], float sum, int nb, int now0, int now1, int fut0,
                         int fut1, const float* __restrict__ vadl, float* __restrict__ probs, float* __restrict__ vad,
                         float* __restrict__ p_now, float* __restrict__ p_future, float* __restrict__ H) {
  const float inv = 1.0f / sum;  // one IEEE division per lane (one per class was VALU-bound)
  const unsigned mnow = ((1u << (now1 - now0 + 1)) - 1u) << now0;
  const unsigned mfut = ((1u << (fut1 - fut0 + 1)) - 1u) << fut0;
  const unsigned bm = (1u << nb) - 1u;
  float h = 0.f, n0 = 0.f, n1 = 0.f, u0 = 0.f, u1 = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x4 p = e[k] * inv;
    *(f32x4*)(probs + f * 256 + 64 * k + 4 * l16) = p;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned c = 64 * k + 4 * l16 + i;
      h += -p[i] * log2f(p[i]);
      const unsigned k0 = c & bm, k1 = (c >> nb) & bm;
      n0 += p[i] * (float)__popc(k0 & mnow);
      n1 += p[i] * (float)__popc(k1 & mnow);
      u0 += p[i] * (float)__popc(k0 & mfut);
      u1 += p[i] * (float)__popc(k1 & mfut);
    }
  }
  h = row_sum16(h);
  n0 = row_sum16(n0);
  n1 = row_sum16(n1);
  u0 = row_sum16(u0);
  u1 = row_sum16(u1);
  if (l16 == 0) {
    H[f] = h;
    const float dn = n0 + n1 + 1e-5f, du = u0 + u1 + 1e-5f;
    p_now[f * 2 + 0] = n0 / dn;
    p_now[f * 2 + 1] = n1 / dn;
    p_future[f * 2 + 0] = u0 / du;
    p_future[f * 2 + 1] = u1 / du;
    vad[f * 2 + 0] = 1.0f / (1.0f + expf(-vadl[f * 2 + 0]));
    vad[f * 2 + 1] = 1.0f / (1.0f + expf(-vadl[f * 2 + 1]));
  }
}

__global__ __launch_bounds__(256) void probs_kernel(const float* __restrict__ logits, const float* __restrict__ vadl,
                                                   int64_t frames, int nb, int now0, int now1, int fut0, int fut1,
                                                   float* __restrict__ probs, float* __restrict__ vad,
                                                   float* __restrict__ p_now, float* __restrict__ p_future,
                                                   float* __restrict__ H) {
  const int l16 = threadIdx.x & 15;
  const int64_t f = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (f >= frames) return;  // row-uniform: the DPP reductions stay inside fully active rows
  f32x4 e[4];
  float mx, sum;
  soft16(logits + f * 256, l16, e, mx, sum);
  probs_frame(f, l16, e, sum, nb, now0, now1, fut0, fut1, vadl, probs, vad, p_now, p_future, H);
}

// ------------------------------------------------------------------------------------------
// get_labels (objective.py:40-76,112-139; integer bit packing, bit-exact for binary VA) and
// loss_vap(reduction='none') (objective.py:220-243) for frames t < T - horizon.
// Lane j < 2*nb owns bit (c = j / nb, bin = j % nb): sequential fp32 window sum / len >= thr.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void labels_loss_kernel(const float* __restrict__ logits, const float* __restrict__ va,
                                                         int B, int Tn, int nl, int4 bf, int nb, float thr,
                                                         int64_t* __restrict__ labels, float* __restrict__ loss) {
  const int l16 = threadIdx.x & 15, row = (threadIdx.x & 63) >> 4;
  const int64_t f = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);  // over B * nl, one 16-lane row each
  if (f >= (int64_t)B * nl) return;
  const int b = (int)(f / nl), t = (int)(f - (int64_t)b * nl);
  const int bfr[4] = {bf.x, bf.y, bf.z, bf.w};
  bool bit = false;
  if (l16 < 2 * nb) {
    const int c = l16 / nb, bin = l16 - c * nb;
    int start = 0;
    for (int i = 0; i < bin; ++i) start += bfr[i];
    const float* p = va + ((int64_t)b * Tn + t + 1 + start) * 2 + c;
    float s = 0.f;
    for (int j = 0; j < bfr[bin]; ++j) s += p[(int64_t)j * 2];
    bit = (s / (float)bfr[bin]) >= thr;
  }
  const unsigned long long m = __ballot(bit);
  // bit index of row lane j = c*nb + bin == j
  const int64_t label = (int64_t)((m >> (16 * row)) & ((1ull << (2 * nb)) - 1ull));
  if (!logits) {
    if (l16 == 0) labels[f] = label;
    return;
  }
  const float* lg = logits + ((int64_t)b * Tn + t) * 256;
  f32x4 e[4];
  float mx, se;
  soft16(lg, l16, e, mx, se);
  if (l16 == 0) {
    labels[f] = label;
    loss[f] = (mx + logf(se)) - lg[label];
  }
}

// probs_kernel plus get_labels (objective.py:40-76,112-139) and loss_vap (reduction none,
// objective.py:220-243) of frames t < nl, in one launch over (16-frame block, clip): the block
// stages the VA probabilities of its frames' projection windows in LDS (va[t] = sigmoid(vad
// logit[t]), the same expression as probs' vad output, so the labels equal those of
// labels_loss_kernel on that output), lane j < 2 nb of a frame's row forms bit j = c nb + bin with
// the same sequential fp32 window sum / len >= thr, a ballot gathers the label, and the loss is
// lse - logit[label] from the softmax's own max / sum.  (A separate labels kernel over 256-frame
// blocks cost 7.5 us per bench step on the tail, before this kernel.)
constexpr int PL_F = 16;  // frames per block: one 16-lane row each
__global__ __launch_bounds__(256) void probs_loss_kernel(const float* __restrict__ logits, const float* __restrict__ vadl,
                                                        int Tn, int nb, int now0, int now1, int fut0, int fut1,
                                                        int4 bf, float thr, float* __restrict__ probs,
                                                        float* __restrict__ vad, float* __restrict__ p_now,
                                                        float* __restrict__ p_future, float* __restrict__ H,
                                                        int64_t* __restrict__ labels, int nl, float* __restrict__ loss) {
  __shared__ float sva[2][PL_F + 128];
  const int b = blockIdx.y, t0 = blockIdx.x * PL_F, tid = threadIdx.x;
  const int bfr[4] = {bf.x, bf.y, bf.z, bf.w};
  int hz = 0;
  for (int i = 0; i < nb; ++i) hz += bfr[i];
  const int l16 = tid & 15, row = tid >> 4, t = t0 + row;
  const int64_t f = (int64_t)b * Tn + t;
  f32x4 e[4];
  if (t < Tn) soft16_load(logits + f * 256, l16, e);  // in flight during the window staging
  const int nrow = min(PL_F + hz, Tn - 1 - t0);  // frames t0 + 1 .. used by this block's windows
  for (int i = tid; i < 2 * nrow; i += 256) {
    const int r = i >> 1, c = i & 1;
    const float x = vadl[((int64_t)b * Tn + t0 + 1 + r) * 2 + c];
    sva[c][r] = 1.0f / (1.0f + expf(-x));
  }
  __syncthreads();
  if (t >= Tn) return;  // row-uniform: the DPP reductions stay inside fully active rows
  float mx, sum;
  soft16_exp(e, mx, sum);
  probs_frame(f, l16, e, sum, nb, now0, now1, fut0, fut1, vadl, probs, vad, p_now, p_future, H);
  bool bit = false;
  if (t < nl && l16 < 2 * nb) {
    const int c = l16 / nb, bin = l16 - c * nb;
    int start = 0;
    for (int i = 0; i < bin; ++i) start += bfr[i];
    float sm = 0.f;
    for (int j = 0; j < bfr[bin]; ++j) sm += sva[c][row + start + j];
    bit = (sm / (float)bfr[bin]) >= thr;
  }
  const unsigned long long m = __ballot(bit);
  if (l16 == 0 && t < nl) {
    const int64_t label = (int64_t)((m >> (16 * (row & 3))) & ((1ull << (2 * nb)) - 1ull));
    const int64_t i = (int64_t)b * nl + t;
    labels[i] = label;
    loss[i] = (mx + logf(sum)) - logits[f * 256 + label];
  }
}

__global__ __launch_bounds__(256) void aggregate_kernel(const float* __restrict__ probs, int64_t frames, int nb,
                                                       int from_bin, int to_bin, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= frames) return;
  const f32x4 p = *(const f32x4*)(probs + f * 256 + lane * 4);
  const unsigned msk = ((1u << (to_bin - from_bin + 1)) - 1u) << from_bin;
  const unsigned bm = (1u << nb) - 1u;
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned k = lane * 4 + i;
    a0 += p[i] * (float)__popc((k & bm) & msk);
    a1 += p[i] * (float)__popc(((k >> nb) & bm) & msk);
  }
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  if (lane == 0) {
    const float d = a0 + a1 + 1e-5f;
    out[f * 2 + 0] = a0 / d;
    out[f * 2 + 1] = a1 / d;
  }
}

// VapGPT.vad (model.py:227-247): sigmoid(vad logits) >= cutoff, then vad_fill_silences / vad_omit_spikes
// (utils.py:239-272; islands via find_island_idx_len :21-49).  One thread per (batch, channel)
// run-length scan; integer semantics, bit-exact.
__global__ void vad_post_kernel(const float* __restrict__ vp, int B, int Tn, float cutoff, int max_fill, int max_omit,
                                float* __restrict__ out) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= 2 * B) return;
  const int b = id >> 1, c = id & 1;
  const float* src = vp + (int64_t)b * Tn * 2 + c;
  float* dst = out + (int64_t)b * Tn * 2 + c;
  for (int t = 0; t < Tn; ++t) dst[(int64_t)t * 2] = (1.0f / (1.0f + expf(-src[(int64_t)t * 2]))) >= cutoff ? 1.f : 0.f;
  for (int pass = 0; pass < 2; ++pass) {
    const float target = pass == 0 ? 0.f : 1.f;  // fill silences (0-runs), then omit spikes (1-runs)
    const int lim = pass == 0 ? max_fill : max_omit;
    int i = 0;
    while (i < Tn) {
      const float v = dst[(int64_t)i * 2];
      int j = i + 1;
      while (j < Tn && dst[(int64_t)j * 2] == v) ++j;
      if (v == target && (j - i) <= lim)
        for (int k = i; k < j; ++k) dst[(int64_t)k * 2] = 1.f - target;
      i = j;
    }
  }
}

template <typename T>
__global__ void convert_kernel(const float* in, T* out, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = from_f32<T>(in[i]);
}
template <typename T>
__global__ void pack_conv_kernel(const float* in, T* out, int N, int C, int KW) {
  const int64_t n = (int64_t)N * C * KW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(i / ((int64_t)C * KW));
    const int rem = (int)(i - (int64_t)o * C * KW);
    const int c = rem / KW, j = rem - c * KW;
    out[(int64_t)o * C * KW + (int64_t)j * C + c] = from_f32<T>(in[i]);
  }
}
__global__ void add_vec_kernel(const float* a, const float* b, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

}  // namespace

template <typename T>
hipError_t launch_conv0(const float* wav, int B, int64_t N, int L0, const float* w0, const float* b0,
                        const float* gamma, const float* beta, T* out, int64_t out_seq_stride, hipStream_t st,
                        int nseq) {
  dim3 grid((L0 + 63) / 64, nseq > 0 ? nseq : 2 * B);
  hipLaunchKernelGGL((conv0_kernel<T>), grid, dim3(256), 0, st, wav, B, N, L0, w0, b0, gamma, beta, out,
                     out_seq_stride);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_zero_rows(T* base, int n_seq, int64_t seq_stride, int rows, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  const int64_t n = (int64_t)rows * 256;
  dim3 grid((unsigned)((n + 255) / 256 < 64 ? (n + 255) / 256 : 64), n_seq);
  hipLaunchKernelGGL((zero_rows_kernel<T>), grid, dim3(256), 0, st, base, seq_stride, rows);
  return hipGetLastError();
}

hipError_t launch_zero_regions(const ZeroRegions& z, int n_seq, hipStream_t st) {
  if (z.n <= 0 || z.n > ZeroRegions::MAX || n_seq <= 0) return hipErrorInvalidValue;
  int64_t most = 0;
  for (int i = 0; i < z.n; ++i) {
    if (z.r[i].bytes % 16 || z.r[i].seq_stride_bytes % 16 || ((uintptr_t)z.r[i].base & 15)) return hipErrorInvalidValue;
    most = std::max<int64_t>(most, z.r[i].bytes / 16);
  }
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(8, (most + 255) / 256)), n_seq, z.n);
  hipLaunchKernelGGL(zero_regions_kernel, grid, dim3(256), 0, st, z);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_layernorm(const float* x, int64_t rows, const float* gamma, const float* beta, float eps, T* out,
                            T* raw, hipStream_t st) {
  hipLaunchKernelGGL((layernorm_kernel<T>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, x, rows, gamma, beta,
                     eps, out, raw);
  return hipGetLastError();
}

hipError_t launch_vad_head(const float* x, int B, int Tn, const float* w, const float* bias, float* vad,
                           hipStream_t st) {
  const int64_t rows = (int64_t)2 * B * Tn;
  hipLaunchKernelGGL(vad_head_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, x, B, Tn, w, bias, vad);
  return hipGetLastError();
}

hipError_t launch_vad_head_rows(const float* x, int64_t x_seq, int B, int Tn, int t0, int nt, const float* w,
                                const float* bias, float* vad, hipStream_t st) {
  if (B <= 0 || nt <= 0 || t0 < 0 || t0 + nt > Tn) return hipErrorInvalidValue;
  const int64_t rows = (int64_t)2 * B * nt;
  hipLaunchKernelGGL(vad_head_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, x, x_seq, B, Tn, t0, nt,
                     w, bias, vad);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_convert_rows(const float* in, int64_t in_seq, T* out, int64_t out_seq, int n_seq, int rows,
                               hipStream_t st) {
  if (n_seq <= 0 || rows <= 0) return hipErrorInvalidValue;
  const int64_t n = (int64_t)n_seq * rows * 64;
  hipLaunchKernelGGL((convert_rows_kernel<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, in_seq, out,
                     out_seq, n_seq, rows);
  return hipGetLastError();
}
template hipError_t launch_convert_rows<float>(const float*, int64_t, float*, int64_t, int, int, hipStream_t);
template hipError_t launch_convert_rows<bf16>(const float*, int64_t, bf16*, int64_t, int, int, hipStream_t);

hipError_t launch_probs(const float* logits, const float* vad_logits, int B, int Tn, int n_bins, int now0, int now1,
                        int fut0, int fut1, float* probs, float* vad, float* p_now, float* p_future, float* H,
                        hipStream_t st) {
  const int64_t frames = (int64_t)B * Tn;
  hipLaunchKernelGGL(probs_kernel, dim3((unsigned)((frames + 15) / 16)), dim3(256), 0, st, logits, vad_logits, frames,
                     n_bins, now0, now1, fut0, fut1, probs, vad, p_now, p_future, H);
  return hipGetLastError();
}

hipError_t launch_labels_loss(const float* logits, const float* va, int B, int Tn, const int* bin_frames, int n_bins,
                              float threshold, int64_t* labels, float* loss, hipStream_t st) {
  if (n_bins < 1 || n_bins > 4) return hipErrorInvalidValue;
  int horizon = 0;
  int4 bf = {0, 0, 0, 0};
  int* bp = &bf.x;
  for (int i = 0; i < n_bins; ++i) {
    bp[i] = bin_frames[i];
    horizon += bin_frames[i];
  }
  const int nl = Tn - horizon;
  if (nl <= 0) return hipErrorInvalidValue;
  const int64_t n = (int64_t)B * nl;
  hipLaunchKernelGGL(labels_loss_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, st, logits, va, B, Tn, nl, bf,
                     n_bins, threshold, labels, loss);
  return hipGetLastError();
}

hipError_t launch_probs_loss(const float* logits, const float* vad_logits, int B, int Tn, int n_bins, int now0,
                             int now1, int fut0, int fut1, const int* bin_frames, float threshold, float* probs,
                             float* vad, float* p_now, float* p_future, float* H, int64_t* labels, float* loss,
                             hipStream_t st) {
  if (n_bins < 1 || n_bins > 4) return hipErrorInvalidValue;
  int horizon = 0;
  int4 bf = {0, 0, 0, 0};
  int* bp = &bf.x;
  for (int i = 0; i < n_bins; ++i) {
    bp[i] = bin_frames[i];
    horizon += bin_frames[i];
  }
  const int nl = Tn - horizon;
  if (nl <= 0 || horizon > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(probs_loss_kernel, dim3((unsigned)((Tn + PL_F - 1) / PL_F), (unsigned)B), dim3(256), 0, st, logits,
                     vad_logits, Tn, n_bins, now0, now1, fut0, fut1, bf, threshold, probs, vad, p_now, p_future, H,
                     labels, nl, loss);
  return hipGetLastError();
}

hipError_t launch_aggregate(const float* probs, int64_t frames, int nb, int from_bin, int to_bin, float* out,
                            hipStream_t st) {
  hipLaunchKernelGGL(aggregate_kernel, dim3((unsigned)((frames + 3) / 4)), dim3(256), 0, st, probs, frames, nb, from_bin,
                     to_bin, out);
  return hipGetLastError();
}
hipError_t launch_vad_post(const float* vad_probs, int B, int Tn, float cutoff, int max_fill, int max_omit, float* out,
                           hipStream_t st) {
  hipLaunchKernelGGL(vad_post_kernel, dim3((2 * B + 63) / 64), dim3(64), 0, st, vad_probs, B, Tn, cutoff, max_fill,
                     max_omit, out);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_convert(const float* in, T* out, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL((convert_kernel<T>), dim3(256), dim3(256), 0, st, in, out, n);
  return hipGetLastError();
}
template <typename T>
hipError_t launch_pack_conv(const float* in, T* out, int N, int C, int KW, hipStream_t st) {
  hipLaunchKernelGGL((pack_conv_kernel<T>), dim3(256), dim3(256), 0, st, in, out, N, C, KW);
  return hipGetLastError();
}
// Packed projection-weight layout (k_rowpanel.hip RowPanelArgs::w_packed, k_ffn.hip): bf16 W [N][K]
// -> [N/256][K/32 k-steps][16 row groups][64 lanes][8], lane = (k%32)/8*16 + n%16: one k-step tile
// of a 256-row N tile is 16 KiB contiguous and one wave's 16-row MFMA fragment 1 KiB.
__global__ void pack_rowpanel_kernel(const chunk16* __restrict__ src, chunk16* __restrict__ dst, int nchunks, int ksteps) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= nchunks) return;
  const int lane = c & 63, grp = (c >> 6) & 15, ks = (c >> 10) % ksteps, nt = (c >> 10) / ksteps;
  const int n = nt * 256 + grp * 16 + (lane & 15), kc = ks * 4 + (lane >> 4);
  dst[c] = src[(int64_t)n * ksteps * 4 + kc];
}
hipError_t launch_pack_rowpanel(const bf16* src, bf16* dst, int N, int K, hipStream_t st) {
  if (N <= 0 || N % 256 || K <= 0 || K % 32) return hipErrorInvalidValue;
  const int nchunks = N * K / 8;
  hipLaunchKernelGGL(pack_rowpanel_kernel, dim3((nchunks + 255) / 256), dim3(256), 0, st, (const chunk16*)src,
                     (chunk16*)dst, nchunks, K / 32);
  return hipGetLastError();
}

hipError_t launch_add_vec(const float* a, const float* b, float* out, int n, hipStream_t st) {
  hipLaunchKernelGGL(add_vec_kernel, dim3((n + 255) / 256), dim3(256), 0, st, a, b, out, n);
  return hipGetLastError();
}

#define INST(T)                                                                                                       \
  template hipError_t launch_conv0<T>(const float*, int, int64_t, int, const float*, const float*, const float*,       \
                                      const float*, T*, int64_t, hipStream_t, int);                                    \
  template hipError_t launch_zero_rows<T>(T*, int, int64_t, int, hipStream_t);                                          \
  template hipError_t launch_layernorm<T>(const float*, int64_t, const float*, const float*, float, T*, T*,           \
                                          hipStream_t);                                                                \
  template hipError_t launch_convert<T>(const float*, T*, int64_t, hipStream_t);                                      \
  template hipError_t launch_pack_conv<T>(const float*, T*, int, int, int, hipStream_t);
INST(float)
INST(bf16)

// ------------------------------------------------------------------------------------------
// VapGPTMono.encode_va (vap/model.py:352-357): LN(va_condition(va) [+ va_cond_history(hist)]),
// added to the encoder output (model.py:378).  One wave per row, 4 channels per lane.
// ------------------------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(256) void va_cond_kernel(float* __restrict__ x, const float* __restrict__ va,
                                                      const float* __restrict__ hist, int rows, int bins,
                                                      const float* __restrict__ Wv, const float* __restrict__ bv,
                                                      const float* __restrict__ Wh, const float* __restrict__ bh,
                                                      const float* __restrict__ gam, const float* __restrict__ bet) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float a0 = va[(int64_t)r * 2], a1 = va[(int64_t)r * 2 + 1];
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = lane * 4 + e;
    float t = fmaf(Wv[c * 2], a0, fmaf(Wv[c * 2 + 1], a1, bv[c]));
    if (hist) {
      t += bh[c];
      for (int k = 0; k < bins; ++k) t = fmaf(Wh[c * bins + k], hist[(int64_t)r * bins + k], t);
    }
    v[e] = t;
  }
  const float mean = wave_sum(v[0] + v[1] + v[2] + v[3]) * (1.0f / 256);
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) ss += (v[e] - mean) * (v[e] - mean);
  const float rstd = rsqrtf(wave_sum(ss) * (1.0f / 256) + 1e-5f);
  float* xr = x + (int64_t)r * 256 + lane * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = lane * 4 + e;
    xr[e] += (v[e] - mean) * rstd * gam[c] + bet[c];
  }
}
}  // namespace

hipError_t launch_va_cond(float* x, const float* va, const float* hist, int rows, int bins, const float* Wv,
                          const float* bv, const float* Wh, const float* bh, const float* gamma, const float* beta,
                          hipStream_t st) {
  if (rows <= 0 || (hist && bins <= 0)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(va_cond_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, va, hist, rows, bins, Wv, bv, Wh, bh,
                     gamma, beta);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Stream-ordered flag hand-offs as kernels (graph-capturable replacements of hipStreamWriteValue32 /
// hipStreamWaitValue32 for the captured streaming push): a store of v to *p after the preceding
// work, and a one-lane bounded spin until *p >= v (~2 s, then the error word is set and the stream
// runs on, so a lost flag never hangs the device).
// ------------------------------------------------------------------------------------------
namespace {
// (the data the flag covers was written by earlier kernels of the stream: their kernel boundary
// wrote it back; the kernels after a wait start behind a boundary too, so neither side needs more
// than agent scope -- and a poll must not be a system-scope acquire: see k_lstm.hip)
__global__ void flag_set_kernel(unsigned* p, unsigned v) {
  if (threadIdx.x == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void wait_geq_kernel(const unsigned* p, unsigned v, unsigned* err) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) {
    __builtin_amdgcn_s_sleep(8);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 100 MHz: 2 s
      if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}
}  // namespace

hipError_t launch_flag_set(unsigned* p, unsigned v, hipStream_t st) {
  hipLaunchKernelGGL(flag_set_kernel, dim3(1), dim3(64), 0, st, p, v);
  return hipGetLastError();
}
hipError_t launch_wait_geq(const unsigned* p, unsigned v, unsigned* err, hipStream_t st) {
  hipLaunchKernelGGL(wait_geq_kernel, dim3(1), dim3(64), 0, st, p, v, err);
  return hipGetLastError();
}
