// Host side of the MI355X VAP engine: parameter store + packing, workspace planning and the
// forward orchestration of VapGPT.forward (vap/model.py:249-268) over HIP kernels.
// Exposes the C ABI declared in include/vap_hip.h.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <tuple>
#include <string>
#include <vector>

#include "../../include/vap_hip.h"
#include "vap_common.h"
#include "vap_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                         \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      return fail(VAP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));           \
  } while (0)

constexpr int D = 256;

struct Param {
  int64_t numel = 0;
  float* dev = nullptr;
  bool set = false;
};

}  // namespace

struct vap_handle {
  vap_dims dims{};
  std::vector<std::string> keys;
  std::map<std::string, Param> params;
  std::map<std::string, void*> packed;  // storage-type buffers
  std::map<std::string, float*> fpacked;  // fp32 derived buffers (e.g. summed LSTM biases)
  bool finalized = false;
  // micro-batch pipeline: side streams for the LSTM recurrences + events
  static constexpr int NSIDE = 3, MAXMB = 16;
  int microbatches = 4;
  // forward: front-end / back-end boundaries (cumulative frame fractions, VAP_TC_FE / VAP_TC_BE;
  // "" = the even time_chunks split for both)
  // (the pair-split recurrence ends well before the caller stream's work: two back-end chunks, the
  // first of 640 frames = 5 full 128-query attention blocks, measured best: 156.2k -> 166.3k audio-s/s)
  // (seven growing front-end pieces started the recurrence sooner in single-forward traces but
  // measured 3.5 % slower in the back-to-back bench: kept as VAP_TC_FE=0.05,0.12,0.2,0.3,0.42,0.56,0.72)
  // (round 3 with the split back end: five pieces 0.12 / 0.3 / 0.5 / 0.7 / 0.85, +0.8 % over the four
  // pieces 0.1 / 0.27 / 0.48 / 0.72 in a same-box A/B: a smaller last piece shortens what the recurrence
  // still has to do after the front end's end)
  std::vector<double> tc_fe{0.12, 0.3, 0.5, 0.7, 0.85}, tc_be{0.64};
  bool tc_be_auto = true;  // back-end chunks of clips longer than 1200 frames by rule (tc_schedule_split)
  bool tc_fe_auto = true;  // + a 120-frame first front-end piece for clips longer than 1200 frames
  bool heads_chunked = true;  // VAP_HEADS_CHUNKED=0: heads once after the last back-end chunk (per chunk,
                              // the fused heads kernel takes the first chunk's heads off the tail after
                              // the recurrence, which binds since the caller stream has ~0.2 ms of slack)
  hipStream_t side[NSIDE] = {};
  // time-pipelined forward: conv2..4 + gate projections of each front-end piece on this high-priority
  // stream while the caller stream runs the next piece's conv01, so each launch's last partial round
  // of workgroups shares the chip with the other kernel (VAP_FE_STREAMS=1: all on the caller stream)
  // (VAP_FE_STREAMS=2, session 4: within 1 % of one stream in the bench, +1.5 % in back-to-back
  // forwards without per-launch timing events; one stream keeps each kernel's events clean)
  int fe_streams = 2;
  hipEvent_t mb_ev[MAXMB] = {};
  hipEvent_t fork_ev[MAXMB] = {};
  int fork_next = 0;
  bool streams_ready = false;
  // persistent-LSTM hand-off (bf16): ready[MAXMB] then done[MAXMB] counters in device memory,
  // monotonic across calls (epoch / cumulative expectations kept here)
  unsigned* sync_mem = nullptr;
  // hand-off error word (1 when a bounded flag wait timed out, so that call's outputs are invalid):
  // host-mapped, so the host reads it without a device sync (vap_forward returns the error on the
  // next call on the handle, vap_synchronize right away)
  unsigned* err_host = nullptr;
  unsigned* err_dev = nullptr;
  // bf16 recurrence: split over workgroup pairs (k_lstm.hip lstm_pair_kernel, two CUs per 16 sequences)
  // conv2..4 on the slab-staged k4 s2 kernel (k_conv234.hip); VAP_CONVK4=0: implicit GEMMs on gemm2
  // time-chunked back end: each layer's block kernel also computes the next layer's LN + Q/K/V (and
  // cross K/V) from the rows it holds, one launch and one read of x less per layer transition
  // (VAP_BLOCK_FUSE=0: separate lnproj launches)
  bool block_fuse = true;
  double be_frac = 0.5;  // VAP_BE_FRAC: clips of the caller stream's group (two groups)
  int be_split = 2;  // VAP_BE_SPLIT=1: the time-chunked back end on the caller stream only (tc_back_end)
  void* xbuf = nullptr;
  size_t xbuf_bytes = 0;
  // exchange tags: every pair-recurrence launch takes the next Tn + 1 values (strictly increasing, so a
  // slot left by any earlier launch never holds a tag a later launch waits for); wraps by clearing xbuf
  unsigned xtag = 0;
  int test_drop_ready = -1;  // tests only (vap_test_drop_ready): never publish ready[c] -> the wait times out
  int lstm_xplain = 0;       // VAP_LSTM_XPLAIN / vap_test_lstm_xplain: pair-exchange store policy (0 = by handshake)
  int lstm_max_wg = 0;  // VAP_LSTM_MAX_WG: persistent recurrence launches at most this many workgroups
  // fp32 parity mode: GEMMs on split-bf16 operands (k_gemm.hip gemm3_kernel; VAP_FP32_EXACT=1: the exact
  // fp32-MFMA kernels); fp32 packed weight -> its split copy [2][N][K] bf16
  bool fp32_split = true;
  bool fp32_quad = true;  // VAP_FP32_QUAD=0: the recurrence on lstm_kernel<float> instead of the quad split
  std::map<const void*, const void*> split_of;
  std::map<std::string, int64_t> packed_numel;
  unsigned epoch = 0;
  unsigned done_expect[MAXMB] = {};
  bool wait_value = false;  // device supports hipStreamWaitValue32 / hipStreamWriteValue32
  int time_chunks = 4;          // VAP_TIME_CHUNKS (bf16, 1-layer LSTM): pipeline the forward along time
  bool use_time_chunks() const {
    return dims.precision == VAP_PRECISION_BF16 && dims.lstm_layers == 1 && time_chunks >= 2 && !dims.mono;
  }
  // VapGPTMono (dims.mono): the VA conditioning inputs of the running vap_forward_mono call
  const float* mono_va = nullptr;
  const float* mono_hist = nullptr;
  int ensure_streams() {
    if (streams_ready) return VAP_OK;
    // side[1] doubles as the front-end stream of the time-pipelined forward (a stream of its own
    // would share one of the process's GPU_MAX_HW_QUEUES hardware queues with another, which
    // measured slower); VAP_FE_PRIO=1 creates it with the highest priority
    int prio_lo = 0, prio_hi = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) return VAP_ERR_HIP;
    for (int i = 0; i < NSIDE; ++i)
      if (hipStreamCreateWithPriority(&side[i], hipStreamNonBlocking, i == 1 ? prio_hi : prio_lo) != hipSuccess)
        return VAP_ERR_HIP;
    for (int i = 0; i < MAXMB; ++i) {
      if (hipEventCreateWithFlags(&mb_ev[i], hipEventDisableTiming) != hipSuccess) return VAP_ERR_HIP;
      if (hipEventCreateWithFlags(&fork_ev[i], hipEventDisableTiming) != hipSuccess) return VAP_ERR_HIP;
    }
    int dev = 0, wv = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, dev) == hipSuccess && wv) {
      if (hipMalloc(&sync_mem, (2 * MAXMB + 1) * sizeof(unsigned)) != hipSuccess) return VAP_ERR_HIP;
      if (hipMemset(sync_mem, 0, (2 * MAXMB + 1) * sizeof(unsigned)) != hipSuccess) return VAP_ERR_HIP;
      if (hipDeviceSynchronize() != hipSuccess) return VAP_ERR_HIP;  // (null stream vs non-blocking side streams)
      if (hipHostMalloc((void**)&err_host, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
          hipHostGetDevicePointer((void**)&err_dev, err_host, 0) != hipSuccess)
        return VAP_ERR_HIP;
      *err_host = 0;
      wait_value = true;
    }
    streams_ready = true;
    return VAP_OK;
  }
  // next fork event of the pool (recorded on the main stream, waited by a side stream); call ONCE
  // per fork and use the returned handle for both the record and the wait
  hipEvent_t next_fork_event() {
    hipEvent_t e = fork_ev[fork_next];
    fork_next = (fork_next + 1) % MAXMB;
    return e;
  }
  // timing hook
  int timing_cls = 0;
  bool timing_serial = false;  // vap_timing(h, -cls): the front end on the caller stream only
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t ev_used = 0;

  ~vap_handle() {
    if (streams_ready) {
      if (sync_mem) (void)hipFree(sync_mem);
      if (err_host) (void)hipHostFree(err_host);
      if (xbuf) (void)hipFree(xbuf);
      for (auto& st : side) (void)hipStreamDestroy(st);
      for (int i = 0; i < MAXMB; ++i) {
        (void)hipEventDestroy(mb_ev[i]);
        (void)hipEventDestroy(fork_ev[i]);
      }
    }
    if (!streams_ready && xbuf) (void)hipFree(xbuf);
    for (auto& kv : params)
      if (kv.second.dev) (void)hipFree(kv.second.dev);
    for (auto& kv : packed) (void)hipFree(kv.second);
    for (auto& kv : fpacked) (void)hipFree(kv.second);
    for (auto& e : ev) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
  }
  const float* P(const std::string& k) const { return params.at(k).dev; }
  template <typename T>
  const T* W(const std::string& k) const { return (const T*)packed.at(k); }
  // attention=True: attention-weight outputs (channel self / cross / cross-layer self), set only for
  // the duration of vap_forward_attention
  float* amap[3] = {nullptr, nullptr, nullptr};
  bool amap_active() const { return amap[0] || amap[1] || amap[2]; }
};

namespace {

static int conv_grid_cap(const vap_handle* h, int S);

void add_schema(vap_handle* h) {
  auto add = [&](const std::string& k, int64_t n) {
    h->keys.push_back(k);
    h->params[k].numel = n;
  };
  const vap_dims& d = h->dims;
  const std::string g = "encoder.encoder.gEncoder";
  const int kws[5] = {10, 8, 4, 4, 4};
  for (int i = 0; i < 5; ++i) {
    const int cin = i == 0 ? 1 : D;
    add(g + ".conv" + std::to_string(i) + ".weight", (int64_t)D * cin * kws[i]);
    add(g + ".conv" + std::to_string(i) + ".bias", D);
    add(g + ".batchNorm" + std::to_string(i) + ".weight", D);
    add(g + ".batchNorm" + std::to_string(i) + ".bias", D);
  }
  for (int l = 0; l < d.lstm_layers; ++l) {
    const std::string p = "encoder.encoder.gAR.baseNet.", s = "_l" + std::to_string(l);
    add(p + "weight_ih" + s, 4 * D * D);
    add(p + "weight_hh" + s, 4 * D * D);
    add(p + "bias_ih" + s, 4 * D);
    add(p + "bias_hh" + s, 4 * D);
  }
  add("encoder.downsample.1.weight", D * D * 5);
  add("encoder.downsample.1.bias", D);
  add("encoder.downsample.2.ln.weight", D);
  add("encoder.downsample.2.ln.bias", D);
  auto layer = [&](const std::string& p, bool cross) {
    add(p + ".ln_self_attn.weight", D);
    add(p + ".ln_self_attn.bias", D);
    add(p + ".ln_ffnetwork.weight", D);
    add(p + ".ln_ffnetwork.bias", D);
    add(p + ".mha.m", d.num_heads);
    for (const char* n : {"key", "query", "value", "proj"}) add(p + ".mha." + n + ".weight", D * D);
    add(p + ".ffnetwork.0.weight", 3 * D * D);
    add(p + ".ffnetwork.3.weight", 3 * D * D);
    if (cross) {
      add(p + ".ln_src_attn.weight", D);
      add(p + ".ln_src_attn.bias", D);
      add(p + ".mha_cross.m", d.num_heads);
      for (const char* n : {"key", "query", "value", "proj"}) add(p + ".mha_cross." + n + ".weight", D * D);
    }
  };
  if (d.mono) {  // VapGPTMono.init_va_conditioning (vap/model.py:317-323)
    add("va_condition.weight", D * 2);
    add("va_condition.bias", D);
    add("va_cond_ln.weight", D);
    add("va_cond_ln.bias", D);
    if (d.va_history_bins > 0) {
      add("va_cond_history.weight", (int64_t)D * d.va_history_bins);
      add("va_cond_history.bias", D);
    }
    for (int l = 0; l < d.channel_layers; ++l) layer("ar_channel.layers." + std::to_string(l), false);
    for (int l = 0; l < d.cross_layers; ++l) layer("ar.layers." + std::to_string(l), false);  // plain GPT
    add("objective.codebook.emb.weight", 256 * 8);
    add("vap_head.weight", 256 * D);
    add("vap_head.bias", 256);
    return;
  }
  for (int l = 0; l < d.channel_layers; ++l) layer("ar_channel.layers." + std::to_string(l), false);
  for (int l = 0; l < d.cross_layers; ++l) layer("ar.layers." + std::to_string(l), true);
  add("ar.combinator.h0_a.weight", D * D);
  add("ar.combinator.h0_b.weight", D * D);
  add("ar.combinator.ln.weight", D);
  add("ar.combinator.ln.bias", D);
  add("objective.codebook.emb.weight", 256 * 8);
  add("va_classifier.weight", D);
  add("va_classifier.bias", 1);
  add("vap_head.weight", 256 * D);
  add("vap_head.bias", 256);
}

int64_t conv_len(int64_t n, int k, int s, int pl, int pr) {
  const int64_t v = n + pl + pr - k;
  return v < 0 ? 0 : v / s + 1;
}

void frame_lengths(int64_t n, int64_t* L) {
  L[0] = conv_len(n, 10, 5, 3, 3);
  L[1] = conv_len(L[0], 8, 4, 2, 2);
  L[2] = conv_len(L[1], 4, 2, 1, 1);
  L[3] = conv_len(L[2], 4, 2, 1, 1);
  L[4] = conv_len(L[3], 4, 2, 1, 1);
  L[5] = conv_len(L[4], 5, 2, 4, 0);
}

// ------------------------------------------------------------------------ workspace plan
struct Plan {
  int B = 0, S = 0, T = 0;
  int64_t L[6]{};
  int64_t s0, s1, s2, s3, s4, sh;  // per-sequence strides (elements) of padded activations
  size_t X0, X1, X2, X3, X4, GX, H0, H1, X, LN, RAW, QKV, KVC, QC, ATT, FF, HC, HCT, total;
  size_t QKVL = 0, KVCL = 0;  // time-chunked mode: Q/K/V (self) and K/V (cross) of EVERY layer are kept
};

size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

Plan make_plan(int B, int64_t N, size_t es, int kv_self_layers = 0, int kv_cross_layers = 0, int ch = 2) {
  Plan p;
  p.B = B;
  p.S = ch * B;  // sequences: 2 speakers per clip (VapGPT), 1 (VapGPTMono)
  frame_lengths(N, p.L);
  p.T = (int)p.L[5];
  const int64_t S = p.S, T = p.T;
  p.s0 = (p.L[0] + 4) * D;
  p.s1 = (p.L[1] + 2) * D;
  p.s2 = (p.L[2] + 2) * D;
  p.s3 = (p.L[3] + 2) * D;
  p.s4 = (p.L[4] + 2) * D;
  p.sh = (p.L[4] + 4) * D;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t r = o;
    o = align_up(o + bytes);
    return r;
  };
  p.X0 = take(es == 2 ? 0 : S * p.s0 * es);  // bf16 mode: conv0 is fused into conv1 (never materialised)
  p.X1 = take(S * p.s1 * es);
  p.X2 = take(S * p.s2 * es);
  p.X3 = take(S * p.s3 * es);
  p.X4 = take(S * p.s4 * es);
  // gate rows: fp32 [S][L4][1024], or bf16 in the pair-recurrence layout (whole groups of 16 sequences)
  p.GX = take(std::max<int64_t>(S * 4, (S + 15) / 16 * 16 * 2) * p.L[4] * 4 * D);
  p.H0 = take(S * p.sh * es);
  p.H1 = take(S * p.sh * es);
  p.X = take(S * T * D * sizeof(float));
  // bf16 mode: LayerNorm, FFN hidden and combinator rows stay on chip (fused row kernels of
  // k_block.hip), so LN / FF / HC / HCT are fp32-mode buffers.  QKV / KVC stay in a time-chunked
  // plan too (its QKVL / KVCL hold every layer's): attention=True and encode run the serial schedule
  const bool fp = es == 4;
  p.LN = take(fp ? S * T * D * es : 0);
  p.RAW = take(S * T * D * es);
  p.QKV = take(S * T * 3 * D * es);
  p.KVC = take(S * T * 2 * D * es);
  p.QC = take(S * T * D * es);
  p.ATT = take(S * T * D * es);
  p.FF = take(fp ? S * T * 3 * D * es : 0);
  p.HC = take(fp ? (size_t)B * T * D * sizeof(float) : 0);
  p.HCT = take(fp ? (size_t)B * T * D * es : 0);
  if (kv_self_layers) p.QKVL = take((size_t)kv_self_layers * S * T * 3 * D * es);
  if (kv_cross_layers) p.KVCL = take((size_t)kv_cross_layers * S * T * 2 * D * es);
  p.total = o;
  return p;
}

Plan plan_for(const vap_handle* h, int B, int64_t N) {
  const size_t es = h->dims.precision == VAP_PRECISION_BF16 ? 2 : 4;
  const int nl = h->dims.channel_layers + h->dims.cross_layers;
  if (h->dims.mono) return make_plan(B, N, es, 0, 0, 1);
  return h->use_time_chunks() ? make_plan(B, N, es, nl, h->dims.cross_layers) : make_plan(B, N, es);
}

// ------------------------------------------------------------------------ timing hook
struct Timed {
  vap_handle* h;
  hipStream_t st;
  bool on;
  size_t idx = 0;
  Timed(vap_handle* hh, int cls, hipStream_t s) : h(hh), st(s), on(hh->timing_cls != 0 && hh->timing_cls == cls) {
    if (!on) return;
    if (h->ev_used == h->ev.size()) {
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      h->ev.push_back({a, b});
    }
    idx = h->ev_used++;
    (void)hipEventRecord(h->ev[idx].first, st);
  }
  ~Timed() {
    if (on) (void)hipEventRecord(h->ev[idx].second, st);
  }
};

template <typename T>
hipError_t gemm(const GemmArgs& g, hipStream_t st, bool out_f32) {
  if (out_f32) return launch_gemm<T, float>(g, st);
  if constexpr (sizeof(T) == 2) return launch_gemm<bf16, bf16>(g, st);
  return launch_gemm<float, float>(g, st);
}

}  // namespace

// fp32 mode: the GEMMs take the split-bf16 copy of their weight (three bf16 MFMAs per tile-step at ~fp32
// accuracy, k_gemm.hip gemm3_kernel) unless the handle runs the exact fp32-MFMA kernels (VAP_FP32_EXACT=1)
template <typename T>
hipError_t hgemm(const vap_handle* h, GemmArgs g, hipStream_t st, bool out_f32);

namespace {

GemmArgs gargs(const void* A, int64_t lda, int64_t aseq, const void* W, int K, int N, const float* bias, int Mps, int nseq,
               void* C, int64_t ldc, int64_t cseq) {
  GemmArgs g{};
  g.A = A;
  g.lda = lda;
  g.a_seq_stride = aseq;
  g.W = W;
  g.K = K;
  g.N = N;
  g.bias = bias;
  g.M_per_seq = Mps;
  g.n_seq = nseq;
  g.C = C;
  g.ldc = ldc;
  g.c_seq_stride = cseq;
  g.eps = 1e-5f;
  return g;
}

// ------------------------------------------------------------------------ packing
uint16_t bf16_bits(float f) {  // round to nearest even
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float bf16_val(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// conv0 with ChannelNorm folded in (see k_conv01.hip): centred weights Wc = W0 - mean_c W0,
// bc = b0 - mean_c b0; MFMA operand rows [g*Wc (hi), g*Wc (hi), g*Wc (lo), g*bc (hi), g*bc (lo)];
// statistics G = Wc^T Wc, h = Wc^T bc, beta = bc.bc.  Computed once in double on the host.
int pack_conv0_fused(vap_handle* h, hipStream_t st) {
  const std::string g = "encoder.encoder.gEncoder";
  std::vector<float> W0(D * 10), b0(D), ga(D);
  HIPCHK(hipMemcpyAsync(W0.data(), h->P(g + ".conv0.weight"), W0.size() * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(b0.data(), h->P(g + ".conv0.bias"), D * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(ga.data(), h->P(g + ".batchNorm0.weight"), D * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  double m[10] = {0}, mb = 0;
  for (int c = 0; c < D; ++c) {
    for (int k = 0; k < 10; ++k) m[k] += W0[c * 10 + k];
    mb += b0[c];
  }
  for (int k = 0; k < 10; ++k) m[k] /= D;
  mb /= D;
  std::vector<double> Wc(D * 10), bc(D);
  for (int c = 0; c < D; ++c) {
    for (int k = 0; k < 10; ++k) Wc[c * 10 + k] = (double)W0[c * 10 + k] - m[k];
    bc[c] = (double)b0[c] - mb;
  }
  std::vector<float> stat(112, 0.f);
  for (int a = 0; a < 10; ++a) {
    for (int b = 0; b < 10; ++b) {
      double acc = 0;
      for (int c = 0; c < D; ++c) acc += Wc[c * 10 + a] * Wc[c * 10 + b];
      stat[a * 10 + b] = (float)acc;
    }
    double acc = 0;
    for (int c = 0; c < D; ++c) acc += Wc[c * 10 + a] * bc[c];
    stat[100 + a] = (float)acc;
  }
  double beta = 0;
  for (int c = 0; c < D; ++c) beta += bc[c] * bc[c];
  stat[110] = (float)beta;
  std::vector<uint16_t> op(D * 32);
  for (int c = 0; c < D; ++c) {
    for (int k = 0; k < 10; ++k) {
      const float wv = (float)(ga[c] * Wc[c * 10 + k]);
      const uint16_t hi = bf16_bits(wv);
      const uint16_t lo = bf16_bits(wv - bf16_val(hi));
      op[c * 32 + k] = hi;
      op[c * 32 + 10 + k] = hi;
      op[c * 32 + 20 + k] = lo;
    }
    const float bv = (float)(ga[c] * bc[c]);
    const uint16_t bh = bf16_bits(bv);
    op[c * 32 + 30] = bh;
    op[c * 32 + 31] = bf16_bits(bv - bf16_val(bh));
  }
  void* dop = nullptr;
  float* dst = nullptr;
  if (hipMalloc(&dop, op.size() * 2) != hipSuccess || hipMalloc(&dst, stat.size() * 4) != hipSuccess)
    return fail(VAP_ERR_HIP, "hipMalloc conv0 operand");
  h->packed["conv0_op"] = dop;
  h->fpacked["conv0_stat"] = dst;
  HIPCHK(hipMemcpyAsync(dop, op.data(), op.size() * 2, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dst, stat.data(), stat.size() * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  return VAP_OK;
}

template <typename T>
int pack_all(vap_handle* h, hipStream_t st) {
  auto alloc = [&](const std::string& name, int64_t n) -> T* {
    void* p = nullptr;
    if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) return nullptr;
    h->packed[name] = p;
    h->packed_numel[name] = n;
    return (T*)p;
  };
  const std::string g = "encoder.encoder.gEncoder";
  const int kws[5] = {10, 8, 4, 4, 4};
  if constexpr (sizeof(T) == 2) {  // fused conv0 operand + ChannelNorm statistics (k_conv01.hip)
    int rc = pack_conv0_fused(h, st);
    if (rc) return rc;
  }
  for (int i = 1; i < 5; ++i) {
    T* w = alloc("conv" + std::to_string(i), (int64_t)D * D * kws[i]);
    if (!w) return fail(VAP_ERR_HIP, "hipMalloc packed conv");
    HIPCHK(launch_pack_conv<T>(h->P(g + ".conv" + std::to_string(i) + ".weight"), w, D, D, kws[i], st));
  }
  if constexpr (sizeof(T) == 2) {  // conv1..4 in the k-step-major layout (conv01's W1 stages, convk4's W)
    for (int i = 1; i < 5; ++i) {
      const std::string c = "conv" + std::to_string(i);
      T* w = alloc(c + "_ks", (int64_t)D * D * kws[i]);
      if (!w) return fail(VAP_ERR_HIP, "hipMalloc packed conv (k-step major)");
      HIPCHK(launch_pack_kstep((const bf16*)h->W<T>(c), (bf16*)w, D, D * kws[i], st));
    }
  }
  for (int l = 0; l < h->dims.lstm_layers; ++l) {
    const std::string p = "encoder.encoder.gAR.baseNet.", s = "_l" + std::to_string(l);
    T* wih = alloc("wih" + s, 4 * D * D);
    float* b = nullptr;
    if (!wih || hipMalloc(&b, 4 * D * sizeof(float)) != hipSuccess) return fail(VAP_ERR_HIP, "hipMalloc lstm");
    h->fpacked["bias" + s] = b;
    if constexpr (sizeof(T) == 2) {  // bf16 pair recurrence: gate scales folded in, rows in gx_wrow order
      HIPCHK(launch_pack_wih_prescaled(h->P(p + "weight_ih" + s), (bf16*)wih, h->P(p + "bias_ih" + s),
                                       h->P(p + "bias_hh" + s), b, st));
      T* whp = alloc("whh_pair" + s, 4 * D * D);  // the pair split's layout (lstm_pair_kernel)
      if (!whp) return fail(VAP_ERR_HIP, "hipMalloc lstm");
      HIPCHK(launch_pack_whh_pair(h->P(p + "weight_hh" + s), (bf16*)whp, st));
    } else {
      T* whh = alloc("whh" + s, 4 * D * D);
      if (!whh) return fail(VAP_ERR_HIP, "hipMalloc lstm");
      HIPCHK(launch_convert<T>(h->P(p + "weight_ih" + s), wih, 4 * D * D, st));
      HIPCHK(launch_pack_whh<T>(h->P(p + "weight_hh" + s), whh, st));
      HIPCHK(launch_add_vec(h->P(p + "bias_ih" + s), h->P(p + "bias_hh" + s), b, 4 * D, st));
      void* wq = nullptr;  // the quad-split recurrence's split-bf16 W_hh (k_lstm.hip lstm_quad_kernel)
      if (hipMalloc(&wq, (size_t)2 * 4 * D * D * sizeof(bf16)) != hipSuccess) return fail(VAP_ERR_HIP, "hipMalloc lstm");
      h->packed["whhq" + s] = wq;
      HIPCHK(launch_pack_whh_quad(h->P(p + "weight_hh" + s), (bf16*)wq, st));
    }
  }
  {
    T* w = alloc("down", D * D * 5);
    if (!w) return fail(VAP_ERR_HIP, "hipMalloc down");
    HIPCHK(launch_pack_conv<T>(h->P("encoder.downsample.1.weight"), w, D, D, 5, st));
  }
  auto cat = [&](const std::string& name, std::vector<std::string> srcs) -> int {
    int64_t total = 0;
    for (auto& k : srcs) total += h->params.at(k).numel;
    T* w = alloc(name, total);
    if (!w) return fail(VAP_ERR_HIP, "hipMalloc " + name);
    int64_t off = 0;
    for (auto& k : srcs) {
      const Param& pr = h->params.at(k);
      HIPCHK(launch_convert<T>(pr.dev, w + off, pr.numel, st));
      off += pr.numel;
    }
    return VAP_OK;
  };
  // bf16: the row-panel projections (K = 256) also get a copy in the packed row-panel layout,
  // "<name>@rp" (one k-step tile 16 KiB contiguous, one wave fragment 1 KiB: k_rowpanel.hip)
  auto rp_copy = [&](const std::string& name, int N, int K = D) -> int {
    if constexpr (sizeof(T) == 2) {
      T* w = alloc(name + "@rp", (int64_t)N * K);
      if (!w) return fail(VAP_ERR_HIP, "hipMalloc " + name + "@rp");
      HIPCHK(launch_pack_rowpanel((const bf16*)h->packed.at(name), (bf16*)w, N, K, st));
    }
    return VAP_OK;
  };
  auto layer = [&](const std::string& p, bool cross) -> int {
    int rc;
    if ((rc = cat(p + ".qkv", {p + ".mha.query.weight", p + ".mha.key.weight", p + ".mha.value.weight"}))) return rc;
    if ((rc = cat(p + ".o", {p + ".mha.proj.weight"}))) return rc;
    if ((rc = cat(p + ".w1", {p + ".ffnetwork.0.weight"}))) return rc;
    if ((rc = cat(p + ".w2", {p + ".ffnetwork.3.weight"}))) return rc;
    if ((rc = rp_copy(p + ".qkv", 3 * D)) || (rc = rp_copy(p + ".o", D)) || (rc = rp_copy(p + ".w1", 3 * D)) ||
        (rc = rp_copy(p + ".w2", D, 3 * D)))
      return rc;
    if (cross) {
      if ((rc = cat(p + ".qc", {p + ".mha_cross.query.weight"}))) return rc;
      if ((rc = cat(p + ".kvc", {p + ".mha_cross.key.weight", p + ".mha_cross.value.weight"}))) return rc;
      if ((rc = cat(p + ".oc", {p + ".mha_cross.proj.weight"}))) return rc;
      if ((rc = rp_copy(p + ".qc", D)) || (rc = rp_copy(p + ".kvc", 2 * D)) || (rc = rp_copy(p + ".oc", D))) return rc;
      if constexpr (sizeof(T) == 2) {  // Q/K/V then cross K/V tiles back to back: the fused block's Wp
        T* w = alloc(p + ".qkvkvc@rp", (int64_t)5 * D * D);
        if (!w) return fail(VAP_ERR_HIP, "hipMalloc " + p + ".qkvkvc@rp");
        HIPCHK(launch_pack_rowpanel((const bf16*)h->packed.at(p + ".qkv"), (bf16*)w, 3 * D, D, st));
        HIPCHK(launch_pack_rowpanel((const bf16*)h->packed.at(p + ".kvc"), (bf16*)w + (int64_t)3 * D * D, 2 * D, D, st));
      }
    }
    return VAP_OK;
  };
  int rc;
  for (int l = 0; l < h->dims.channel_layers; ++l)
    if ((rc = layer("ar_channel.layers." + std::to_string(l), false))) return rc;
  for (int l = 0; l < h->dims.cross_layers; ++l)
    if ((rc = layer("ar.layers." + std::to_string(l), !h->dims.mono))) return rc;
  if (!h->dims.mono) {
    if ((rc = cat("comb_a", {"ar.combinator.h0_a.weight"}))) return rc;
    if ((rc = cat("comb_b", {"ar.combinator.h0_b.weight"}))) return rc;
    if ((rc = rp_copy("comb_a", D)) || (rc = rp_copy("comb_b", D))) return rc;  // fused heads (k_block.hip)
  }
  if ((rc = cat("head", {"vap_head.weight"}))) return rc;
  if (!h->dims.mono && (rc = rp_copy("head", 256))) return rc;
  if constexpr (sizeof(T) == 4) {  // split-bf16 copies of every GEMM weight (not W_hh: the recurrence packs its own)
    std::vector<std::pair<std::string, int64_t>> todo;
    for (auto& kv : h->packed_numel)
      if (kv.first.rfind("whh", 0) != 0) todo.push_back(kv);
    for (auto& kv : todo) {
      const std::string& n = kv.first;  // the GEMM's K (the weight's row length) by weight
      const int K = n.rfind("conv", 0) == 0 ? kws[n[4] - '0'] * D : n == "down" ? 5 * D
                    : (n.size() > 3 && n.compare(n.size() - 3, 3, ".w2") == 0) ? 3 * D : D;
      void* sp = nullptr;
      if (hipMalloc(&sp, kv.second * 2 * sizeof(bf16)) != hipSuccess) return fail(VAP_ERR_HIP, "hipMalloc split weight");
      h->packed[kv.first + "@s"] = sp;
      HIPCHK(launch_split_bf16((const float*)h->packed.at(kv.first), (bf16*)sp, kv.second, K, st));
      h->split_of[h->packed.at(kv.first)] = sp;
    }
  }
  return VAP_OK;
}

}  // namespace

template <typename T>
hipError_t hgemm(const vap_handle* h, GemmArgs g, hipStream_t st, bool out_f32) {
  if constexpr (sizeof(T) == 4) {
    if (h->fp32_split) {
      auto it = h->split_of.find(g.W);
      if (it != h->split_of.end()) {
        g.W = it->second;
        g.split = 1;
      }
    }
  }
  return gemm<T>(g, st, out_f32);
}

namespace {

// ------------------------------------------------------------------------ forward
// Sequences are CLIP-MAJOR: seq s = 2*clip + channel (speaker), matching the [B][2][N] waveform,
// so a micro-batch of clips is one contiguous sequence range, and the stereo partner of s is s^1.
struct Range {
  int c0, nc;  // clips [c0, c0+nc)
  int ch = 2;  // sequences per clip (1: VapGPTMono)
  int s0() const { return ch * c0; }
  int ns() const { return ch * nc; }
};

// bf16 transformer layer on row-panel kernels: LayerNorm fused into the A-panel load of the
// Q/K/V, cross-Q and FFN-up projections; residual adds fused into the output projections.
// attention weights of layer `layer` (attention=True only): which = 0 channel self, 1 cross, 2 cross self
template <typename T>
int attn_maps(vap_handle* h, const AttnArgs& a, int which, int layer, Range r, hipStream_t st) {
  if (!h->amap[which]) return VAP_OK;
  const int L = which == 0 ? h->dims.channel_layers : h->dims.cross_layers;
  const int64_t TT = (int64_t)a.T * a.T, per_seq = (int64_t)L * a.H * TT;
  float* out = h->amap[which] + (int64_t)r.s0() * per_seq + (int64_t)layer * a.H * TT;
  HIPCHK(launch_attn_probs<T>(a, out, per_seq, TT, st));
  return VAP_OK;
}

// bf16 transformer layer (modules.py:246-275) on the fused row kernels of k_block.hip, over the
// contiguous rows of a clip range:
//   lnproj: LN_self + Q/K/V (+ the raw-row cross K/V: modules.py:265-272 take the UN-normalised x)
//   attn3:  self attention;  [stereo] lnproj: out-proj + residual + LN_src + cross Q;  attn3: cross
//   block:  last out-projection + residual + LN + FFN + residual
int tr_layer_bf16(vap_handle* h, const Plan& p, unsigned char* ws, const std::string& pre, bool cross, Range r,
                  hipStream_t st, int layer) {
  using T = bf16;
  const int T_ = p.T;
  const int S = r.ns();
  const int rows = S * T_;
  const int64_t so = (int64_t)r.s0() * T_;
  float* X = (float*)(ws + p.X) + so * D;
  T* QKV = (T*)(ws + p.QKV) + so * 3 * D;
  T* KVC = (T*)(ws + p.KVC) + so * 2 * D;
  T* QC = (T*)(ws + p.QC) + so * D;
  T* ATT = (T*)(ws + p.ATT) + so * D;
  const int H = h->dims.num_heads;
  const float scale = 1.0f / std::sqrt((float)D);
  const int64_t t1 = (int64_t)T_ * D, t2 = 2 * t1, t3 = 3 * t1;
  auto lnp = [&](const T* o, const std::string& wo, const std::string& wp, int np, T* cp, int64_t ldp,
                 const std::string& wr, int nr, T* cr, int64_t ldr, const std::string& ln) {
    LnProjArgs a{};
    a.x = X; a.o = o; a.M = rows; a.rows_per_seq = 0; a.x_seq = t1; a.o_seq = t1;
    a.Wo = o ? h->W<T>(wo + "@rp") : nullptr; a.Wp = h->W<T>(wp + "@rp"); a.Wr = nr ? h->W<T>(wr + "@rp") : nullptr;
    a.cp = cp; a.ldp = ldp; a.cp_seq = (int64_t)T_ * ldp; a.cr = cr; a.ldr = ldr; a.cr_seq = (int64_t)T_ * ldr;
    a.gamma = h->P(ln + ".weight"); a.beta = h->P(ln + ".bias"); a.eps = 1e-5f; a.np = np; a.nr = nr;
    return launch_lnproj(a, st);
  };
  {
    Timed tm(h, VAP_K_TR_GEMM, st);
    HIPCHK(lnp(nullptr, "", pre + ".qkv", 3, QKV, 3 * D, pre + ".kvc", cross ? 2 : 0, KVC, 2 * D, pre + ".ln_self_attn"));
  }
  {
    Timed tm(h, VAP_K_ATTN, st);
    AttnArgs a{QKV, 3 * D, t3, QKV + D, 3 * D, t3, QKV + 2 * D, 3 * D, t3, ATT, D, t1, h->P(pre + ".mha.m"), S, T_, H,
               0, scale};
    HIPCHK(launch_attention<T>(a, st));
    if (int rc = attn_maps<T>(h, a, cross ? 2 : 0, layer, r, st)) return rc;
  }
  if (cross) {
    {
      Timed tm(h, VAP_K_TR_GEMM, st);
      HIPCHK(lnp(ATT, pre + ".o", pre + ".qc", 1, QC, D, "", 0, nullptr, 0, pre + ".ln_src_attn"));
    }
    {
      Timed tm(h, VAP_K_ATTN, st);
      AttnArgs a{QC, D, t1, KVC, 2 * D, t2, KVC + D, 2 * D, t2, ATT, D, t1, h->P(pre + ".mha_cross.m"), S, T_, H, 1,
                 scale};
      HIPCHK(launch_attention<T>(a, st));
      if (int rc = attn_maps<T>(h, a, 1, layer, r, st)) return rc;
    }
  }
  {
    Timed tm(h, VAP_K_TR_GEMM, st);
    BlockArgs b{X, ATT, rows, 0, 0, 0, h->W<T>(pre + (cross ? ".oc@rp" : ".o@rp")), h->W<T>(pre + ".w1@rp"),
                h->W<T>(pre + ".w2@rp"), h->P(pre + ".ln_ffnetwork.weight"), h->P(pre + ".ln_ffnetwork.bias"), 1e-5f};
    HIPCHK(launch_block(b, 0, st));
  }
  return VAP_OK;
}

template <typename T>
int tr_layer(vap_handle* h, const Plan& p, unsigned char* ws, const std::string& pre, bool cross, Range r,
             hipStream_t st, int layer) {
  if constexpr (sizeof(T) == 2) return tr_layer_bf16(h, p, ws, pre, cross, r, st, layer);
  const int T_ = p.T;
  const int S = r.ns();
  const int64_t rows = (int64_t)S * T_;
  const int64_t so = (int64_t)r.s0() * T_;  // row offset of the range
  float* X = (float*)(ws + p.X) + so * D;
  T* LN = (T*)(ws + p.LN) + so * D;
  T* RAW = (T*)(ws + p.RAW) + so * D;
  T* QKV = (T*)(ws + p.QKV) + so * 3 * D;
  T* KVC = (T*)(ws + p.KVC) + so * 2 * D;
  T* QC = (T*)(ws + p.QC) + so * D;
  T* ATT = (T*)(ws + p.ATT) + so * D;
  T* FF = (T*)(ws + p.FF) + so * 3 * D;
  const int H = h->dims.num_heads;
  const float scale = 1.0f / std::sqrt((float)D);
  const int64_t t1 = (int64_t)T_ * D, t2 = 2 * t1, t3 = 3 * t1;
  auto resid = [&](GemmArgs g) {
    g.add = X;
    g.ld_add = D;
    g.add_seq_stride = t1;
    return g;
  };
  {
    Timed tm(h, VAP_K_NORM, st);
    HIPCHK(launch_layernorm<T>(X, rows, h->P(pre + ".ln_self_attn.weight"), h->P(pre + ".ln_self_attn.bias"), 1e-5f, LN,
                               cross ? RAW : nullptr, st));
  }
  {
    Timed tm(h, VAP_K_TR_GEMM, st);
    HIPCHK(hgemm<T>(h, gargs(LN, D, t1, h->W<T>(pre + ".qkv"), D, 3 * D, nullptr, T_, S, QKV, 3 * D, t3), st, false));
    if (cross)  // K/V of the cross attention come from the UN-normalised pre-layer x (modules.py:265-272)
      HIPCHK(hgemm<T>(h, gargs(RAW, D, t1, h->W<T>(pre + ".kvc"), D, 2 * D, nullptr, T_, S, KVC, 2 * D, t2), st, false));
  }
  {
    Timed tm(h, VAP_K_ATTN, st);
    AttnArgs a{QKV, 3 * D, t3, QKV + D, 3 * D, t3, QKV + 2 * D, 3 * D, t3, ATT, D, t1, h->P(pre + ".mha.m"), S, T_, H,
               0, scale};
    a.split = h->fp32_split ? 1 : 0;
    HIPCHK(launch_attention<T>(a, st));
    if (int rc = attn_maps<T>(h, a, cross ? 2 : 0, layer, r, st)) return rc;
  }
  {
    Timed tm(h, VAP_K_TR_GEMM, st);
    HIPCHK(hgemm<T>(h, resid(gargs(ATT, D, t1, h->W<T>(pre + ".o"), D, D, nullptr, T_, S, X, D, t1)), st, true));
  }
  if (cross) {
    {
      Timed tm(h, VAP_K_NORM, st);
      HIPCHK(launch_layernorm<T>(X, rows, h->P(pre + ".ln_src_attn.weight"), h->P(pre + ".ln_src_attn.bias"), 1e-5f, LN,
                                 nullptr, st));
    }
    {
      Timed tm(h, VAP_K_TR_GEMM, st);
      HIPCHK(hgemm<T>(h, gargs(LN, D, t1, h->W<T>(pre + ".qc"), D, D, nullptr, T_, S, QC, D, t1), st, false));
    }
    {
      Timed tm(h, VAP_K_ATTN, st);
      AttnArgs a{QC, D, t1, KVC, 2 * D, t2, KVC + D, 2 * D, t2, ATT, D, t1, h->P(pre + ".mha_cross.m"), S, T_, H, 1,
                 scale};
      a.split = h->fp32_split ? 1 : 0;
      HIPCHK(launch_attention<T>(a, st));
      if (int rc = attn_maps<T>(h, a, 1, layer, r, st)) return rc;
    }
    {
      Timed tm(h, VAP_K_TR_GEMM, st);
      HIPCHK(hgemm<T>(h, resid(gargs(ATT, D, t1, h->W<T>(pre + ".oc"), D, D, nullptr, T_, S, X, D, t1)), st, true));
    }
  }
  {
    Timed tm(h, VAP_K_NORM, st);
    HIPCHK(launch_layernorm<T>(X, rows, h->P(pre + ".ln_ffnetwork.weight"), h->P(pre + ".ln_ffnetwork.bias"), 1e-5f, LN,
                               nullptr, st));
  }
  {
    Timed tm(h, VAP_K_TR_GEMM, st);
    GemmArgs g = gargs(LN, D, t1, h->W<T>(pre + ".w1"), D, 3 * D, nullptr, T_, S, FF, 3 * D, t3);
    g.act = 2;
    HIPCHK(hgemm<T>(h, g, st, false));
    HIPCHK(hgemm<T>(h, resid(gargs(FF, 3 * D, t3, h->W<T>(pre + ".w2"), 3 * D, D, nullptr, T_, S, X, D, t1)), st, true));
  }
  return VAP_OK;
}

// Front end of a clip range: conv0..conv4 (+ChannelNorm+ReLU) and the LSTM input projection of
// layer 0.  All on `st`.
template <typename T>
int front_end(vap_handle* h, const Plan& p, const float* wav, int64_t N, unsigned char* ws, Range r, hipStream_t st) {
  const int S = r.ns();
  const int64_t* L = p.L;
  const std::string g = "encoder.encoder.gEncoder";
  T* X0 = (T*)(ws + p.X0) + r.s0() * p.s0;
  T* Xs[4] = {(T*)(ws + p.X1) + r.s0() * p.s1, (T*)(ws + p.X2) + r.s0() * p.s2, (T*)(ws + p.X3) + r.s0() * p.s3,
              (T*)(ws + p.X4) + r.s0() * p.s4};
  const int64_t ss[4] = {p.s1, p.s2, p.s3, p.s4};
  int first = 0;
  if constexpr (sizeof(T) == 2) {  // fused conv0 -> CN0 -> ReLU -> conv1 -> CN1 -> ReLU (k_conv01.hip)
    Timed tm(h, VAP_K_CONV1, st);
    HIPCHK(launch_conv01(wav + (int64_t)r.s0() * N, S, N, (int)L[0], (int)L[1], (const bf16*)h->W<T>("conv0_op"),
                         h->fpacked.at("conv0_stat"), h->P(g + ".batchNorm0.bias"), (const bf16*)h->W<T>("conv1"), (const bf16*)h->W<T>("conv1_ks"),
                         h->P(g + ".conv1.bias"), h->P(g + ".batchNorm1.weight"), h->P(g + ".batchNorm1.bias"),
                         (bf16*)(Xs[0] + D), p.s1, st));
    first = 1;
  } else {  // conv0 + CN0 + ReLU  (encoder_components.py:99), then conv1 as an implicit GEMM
    Timed tm(h, VAP_K_CONV0, st);
    HIPCHK(launch_conv0<T>(wav + (int64_t)r.s0() * N, r.nc, N, (int)L[0], h->P(g + ".conv0.weight"),
                           h->P(g + ".conv0.bias"), h->P(g + ".batchNorm0.weight"), h->P(g + ".batchNorm0.bias"), X0,
                           p.s0, st, S));
  }
  // conv1..conv4 as implicit GEMMs with ChannelNorm + ReLU epilogue (encoder_components.py:100-103)
  const T* ins[4] = {X0, Xs[0], Xs[1], Xs[2]};
  const int64_t in_ss[4] = {p.s0, p.s1, p.s2, p.s3};
  const int lda[4] = {4 * D, 2 * D, 2 * D, 2 * D};
  const int Ks[4] = {8 * D, 4 * D, 4 * D, 4 * D};
  for (int i = first; i < 4; ++i) {
    const std::string c = std::to_string(i + 1);
    Timed tm(h, i == 0 ? VAP_K_CONV1 : VAP_K_CONV234, st);
    if constexpr (sizeof(T) == 2) {
      if (i >= 1) {
        ConvK4Args ca{(const bf16*)ins[i], in_ss[i], (int)(in_ss[i] / D), (const bf16*)h->W<T>("conv" + c + "_ks"),
                      h->P(g + ".conv" + c + ".bias"), h->P(g + ".batchNorm" + c + ".weight"),
                      h->P(g + ".batchNorm" + c + ".bias"), (bf16*)(Xs[i] + D), ss[i], (int)L[i + 1]};
        ca.grid_cap = conv_grid_cap(h, S);
        HIPCHK(launch_convk4(ca, S, st));
        continue;
      }
    }
    GemmArgs ga = gargs(ins[i], lda[i], in_ss[i], h->W<T>("conv" + c), Ks[i], D, h->P(g + ".conv" + c + ".bias"),
                        (int)L[i + 1], S, Xs[i] + D, D, ss[i]);
    ga.norm = 1;
    ga.act = 1;
    ga.gamma = h->P(g + ".batchNorm" + c + ".weight");
    ga.beta = h->P(g + ".batchNorm" + c + ".bias");
    HIPCHK(hgemm<T>(h, ga, st, false));
  }
  return VAP_OK;
}

int launch_rec(vap_handle* h, const bf16* GX, int seq0, int S, int L4, int layer, bf16* out, int64_t out_stride,
               hipStream_t st, const LstmSync* sy, int xg0);
int launch_rec_f32(vap_handle* h, const float* GX, int S, int L4, int layer, float* out, int64_t out_stride,
                   hipStream_t st, int xg0);

// LSTM layer l of a clip range: input projection GEMM on `st`, recurrence on `rec_st`
// (bf16 mode: gx bf16, W_hh resident on the CU).
template <typename T>
int lstm_layer(vap_handle* h, const Plan& p, unsigned char* ws, int l, Range r, hipStream_t st, hipStream_t rec_st,
               bool recurrence = true, int xg0 = 0) {
  const int S = r.ns();
  const int64_t L4 = p.L[4];
  const std::string s = "_l" + std::to_string(l);
  T* X4 = (T*)(ws + p.X4) + r.s0() * p.s4;
  T* Hb[2] = {(T*)(ws + p.H0) + r.s0() * p.sh, (T*)(ws + p.H1) + r.s0() * p.sh};
  constexpr bool bf = sizeof(T) == 2;
  // bf16: the whole batch's gate buffer in the pair-recurrence layout, this range from sequence r.s0()
  void* GX = bf ? (void*)(ws + p.GX) : (void*)((float*)(ws + p.GX) + r.s0() * L4 * 4 * D);
  const T* in = l == 0 ? X4 + D : Hb[(l - 1) & 1] + 4 * D;
  const int64_t in_seq = l == 0 ? p.s4 : p.sh;
  {
    Timed tm(h, VAP_K_LSTM_PROJ, st);
    GemmArgs ga = gargs(in, D, in_seq, h->W<T>("wih" + s), D, 4 * D, h->fpacked.at("bias" + s), (int)L4, S, GX, 4 * D,
                        L4 * 4 * D);
    if (bf) {
      ga.c_pair = 1;
      ga.c_s0 = r.s0();
      ga.c_tn = (int)L4;
    }
    HIPCHK(hgemm<T>(h, ga, st, !bf));
  }
  if (!recurrence) return VAP_OK;
  if (rec_st != st) {  // fork: the recurrence waits for the projection (ONE event from the pool)
    hipEvent_t fork = h->next_fork_event();
    HIPCHK(hipEventRecord(fork, st));
    HIPCHK(hipStreamWaitEvent(rec_st, fork, 0));
  }
  {
    Timed tm(h, VAP_K_LSTM_REC, rec_st);
    if constexpr (bf) {
      if (int rc = launch_rec(h, (const bf16*)GX, r.s0(), S, (int)L4, l, (bf16*)(Hb[l & 1] + 4 * D), p.sh, rec_st, nullptr,
                              xg0))
        return rc;
    } else if (h->fp32_split && h->fp32_quad) {
      if (int rc = launch_rec_f32(h, (const float*)GX, S, (int)L4, l, (float*)(Hb[l & 1] + 4 * D), p.sh, rec_st, xg0))
        return rc;
    } else
      HIPCHK(launch_lstm<T>((const float*)GX, S, (int)L4, h->W<T>("whh" + s), Hb[l & 1] + 4 * D, p.sh, rec_st));
  }
  return VAP_OK;
}

// Combinator (modules.py:434-449) + heads (model.py:257-261) of a clip range, from the final
// residual stream X.  On `st`.
template <typename T>
int heads(vap_handle* h, const Plan& p, unsigned char* ws, Range r, float* logits, float* vadl, hipStream_t st,
          bool raw_ready = false) {
  const int S = r.ns(), T_ = p.T;
  const int64_t t1 = (int64_t)T_ * D;
  float* X = (float*)(ws + p.X) + r.s0() * t1;
  T* RAW = (T*)(ws + p.RAW) + r.s0() * t1;
  if (h->dims.mono) {  // VapGPTMono: logits = vap_head(x) (vap/model.py:384-385); no combinator / VAD head
    Timed tm(h, VAP_K_HEADS, st);
    HIPCHK(launch_layernorm<T>(X, (int64_t)S * T_, nullptr, nullptr, 0.f, nullptr, RAW, st));  // fp32 -> storage
    HIPCHK(hgemm<T>(h, gargs(RAW, D, t1, h->W<T>("head"), D, 256, h->P("vap_head.bias"), T_, S,
                         logits + (int64_t)r.c0 * T_ * 256, 256, (int64_t)T_ * 256), st, true));
    return VAP_OK;
  }
  float* HC = (float*)(ws + p.HC) + r.c0 * t1;
  T* HCT = (T*)(ws + p.HCT) + r.c0 * t1;
  if constexpr (sizeof(T) == 2) {
    {  // combinator + vap_head + va_classifier in one launch (k_block.hip heads_kernel)
      Timed tm(h, VAP_K_HEADS, st);
      if (!raw_ready) HIPCHK(launch_layernorm<T>(X, (int64_t)S * T_, nullptr, nullptr, 0.f, nullptr, RAW, st));
      HeadsArgs ha{(const bf16*)RAW, t1, r.nc * T_, T_, (const bf16*)h->W<T>("comb_a@rp"), (const bf16*)h->W<T>("comb_b@rp"),
                   (const bf16*)h->W<T>("head@rp"), h->P("ar.combinator.ln.weight"), h->P("ar.combinator.ln.bias"),
                   h->P("vap_head.bias"), logits + r.c0 * (int64_t)T_ * 256, 1e-5f, h->P("va_classifier.weight"),
                   h->P("va_classifier.bias"), vadl + r.c0 * (int64_t)T_ * 2};
      ha.xf = X;
      HIPCHK(launch_heads(ha, st));
      return VAP_OK;
    }
  }
  {
    Timed tm(h, VAP_K_HEADS, st);
    if (!raw_ready) HIPCHK(launch_layernorm<T>(X, (int64_t)S * T_, nullptr, nullptr, 0.f, nullptr, RAW, st));
    // channel-0 rows are the even sequences: stride 2*T*D over the clips of the range
    GemmArgs ga = gargs(RAW, D, 2 * t1, h->W<T>("comb_a"), D, D, nullptr, T_, r.nc, HC, D, t1);
    ga.norm = 2;
    ga.act = 2;
    ga.gamma = h->P("ar.combinator.ln.weight");
    ga.beta = h->P("ar.combinator.ln.bias");
    HIPCHK(hgemm<T>(h, ga, st, true));
    // second half + the first's fp32 rows, stored straight in the storage type (the vap_head GEMM's
    // operand; a separate fp32 -> bf16 pass over HC cost 16 us per bench step)
    GemmArgs gb = ga;
    gb.A = RAW + t1;
    gb.W = h->W<T>("comb_b");
    gb.add = HC;
    gb.ld_add = D;
    gb.add_seq_stride = t1;
    gb.C = HCT;
    HIPCHK(hgemm<T>(h, gb, st, false));
    HIPCHK(hgemm<T>(h, gargs(HCT, D, t1, h->W<T>("head"), D, 256, h->P("vap_head.bias"), T_, r.nc,
                         logits + r.c0 * (int64_t)T_ * 256, 256, (int64_t)T_ * 256), st, true));
    HIPCHK(launch_vad_head(X, r.nc, T_, h->P("va_classifier.weight"), h->P("va_classifier.bias"),
                           vadl + r.c0 * (int64_t)T_ * 2, st));
  }
  return VAP_OK;
}


// Back end of a clip range: downsample, transformer stack, combinator, heads.  On `st`.
template <typename T>
int back_end(vap_handle* h, const Plan& p, unsigned char* ws, Range r, float* logits, float* vadl, float* enc_out,
             hipStream_t st) {
  const int S = r.ns(), T_ = p.T;
  const int NL = h->dims.lstm_layers;
  const int64_t t1 = (int64_t)T_ * D;
  T* Hf = (T*)(ws + ((NL - 1) & 1 ? p.H1 : p.H0)) + r.s0() * p.sh;
  float* X = (float*)(ws + p.X) + r.s0() * t1;
  {  // downsample: CConv1d k5 s2 causal + LayerNorm + GELU (encoder_components.py:485-499)
    Timed tm(h, VAP_K_DOWNSAMPLE, st);
    GemmArgs ga = gargs(Hf, 2 * D, p.sh, h->W<T>("down"), 5 * D, D, h->P("encoder.downsample.1.bias"), T_, S, X, D, t1);
    ga.norm = 2;
    ga.act = 2;
    ga.gamma = h->P("encoder.downsample.2.ln.weight");
    ga.beta = h->P("encoder.downsample.2.ln.bias");
    HIPCHK(hgemm<T>(h, ga, st, true));
  }
  if (enc_out) {  // EncoderCPC output, (x1, x2) = channel 0 / 1 -> enc_out [2][B][T][256] ([B][T][256] mono)
    const int64_t B = p.B;
    for (int c = 0; c < r.ch; ++c)
      HIPCHK(hipMemcpy2DAsync(enc_out + ((int64_t)c * B + r.c0) * t1, t1 * sizeof(float), X + c * t1,
                              r.ch * t1 * sizeof(float), t1 * sizeof(float), r.nc, hipMemcpyDeviceToDevice, st));
    return VAP_OK;
  }
  if (h->dims.mono) {  // x = x + encode_va(va, va_history) (vap/model.py:352-357, 378)
    Timed tm(h, VAP_K_NORM, st);
    const int bins = h->dims.va_history_bins;
    const bool hist = bins > 0 && h->mono_hist;
    HIPCHK(launch_va_cond(X, h->mono_va + (int64_t)r.c0 * T_ * 2, hist ? h->mono_hist + (int64_t)r.c0 * T_ * bins : nullptr,
                          S * T_, bins, h->P("va_condition.weight"), h->P("va_condition.bias"),
                          hist ? h->P("va_cond_history.weight") : nullptr, hist ? h->P("va_cond_history.bias") : nullptr,
                          h->P("va_cond_ln.weight"), h->P("va_cond_ln.bias"), st));
  }
  int rc;
  for (int l = 0; l < h->dims.channel_layers; ++l)
    if ((rc = tr_layer<T>(h, p, ws, "ar_channel.layers." + std::to_string(l), false, r, st, l))) return rc;
  for (int l = 0; l < h->dims.cross_layers; ++l)
    if ((rc = tr_layer<T>(h, p, ws, "ar.layers." + std::to_string(l), !h->dims.mono, r, st, l))) return rc;

  return heads<T>(h, p, ws, r, logits, vadl, st);
}

// ------------------------------------------------------------------------ time-chunked forward
// bf16 transformer layer on frames [f0, f1) of EVERY sequence (time-chunked back end).  The layer's
// Q/K/V (self) and K/V (cross) live in per-layer buffers so later chunks attend to earlier ones:
// attention is causal, so queries [f0, f1) need keys [0, f1) only (modules.py:169-202).
// With a next layer (`next` non-empty: its name, `ncross` whether it has cross attention) the block
// kernel also writes that layer's Q/K/V and cross K/V rows; `projected`: this layer's were written so.
int tr_layer_tc(vap_handle* h, const Plan& p, unsigned char* ws, const std::string& pre, bool cross, int li, int ci,
                int f0, int f1, hipStream_t st, bf16* xb_out = nullptr, bool projected = false,
                const std::string& next = "", bool ncross = false, int s0 = 0, int sn = -1) {
  // sequences [s0, s0 + sn) only (s0 even: cross attention pairs s with s ^ 1); layer strides stay p.S
  using T = bf16;
  const int T_ = p.T, S = sn < 0 ? p.S : sn, nf = f1 - f0;
  const int64_t t1 = (int64_t)T_ * D, t2 = 2 * t1, t3 = 3 * t1;
  float* X = (float*)(ws + p.X) + (int64_t)s0 * t1;
  T* QKV = (T*)(ws + p.QKVL) + (int64_t)li * p.S * t3 + (int64_t)s0 * t3;
  T* KVC = (T*)(ws + p.KVCL) + (int64_t)ci * p.S * t2 + (int64_t)s0 * t2;
  T* QC = (T*)(ws + p.QC) + (int64_t)s0 * t1;
  T* ATT = (T*)(ws + p.ATT) + (int64_t)s0 * t1;
  if (xb_out) xb_out += (int64_t)s0 * t1;
  const int H = h->dims.num_heads;
  const float scale = 1.0f / std::sqrt((float)D);
  float* Xf = X + (int64_t)f0 * D;
  // fused LN projections (k_block.hip): rows (s, t in [f0, f1)), x / o / outputs at row f0 of sequence 0
  auto lnp = [&](const T* o, const std::string& wo, const std::string& wp, int np, T* cp, int64_t ldp, int64_t cpseq,
                 const std::string& wr, int nr, T* cr, int64_t ldr, int64_t crseq, const std::string& ln) {
    LnProjArgs a{};
    a.x = Xf; a.o = o; a.M = S * nf; a.rows_per_seq = nf; a.x_seq = t1; a.o_seq = t1;
    a.Wo = o ? h->W<T>(wo + "@rp") : nullptr; a.Wp = h->W<T>(wp + "@rp"); a.Wr = nr ? h->W<T>(wr + "@rp") : nullptr;
    a.cp = cp; a.ldp = ldp; a.cp_seq = cpseq; a.cr = cr; a.ldr = ldr; a.cr_seq = crseq;
    a.gamma = h->P(ln + ".weight"); a.beta = h->P(ln + ".bias"); a.eps = 1e-5f; a.np = np; a.nr = nr;
    return launch_lnproj(a, st);
  };
  if (!projected) {
    Timed tm(h, VAP_K_TR_GEMM, st);  // LN + QKV and the raw-row cross K/V from one read of x
    HIPCHK(lnp(nullptr, "", pre + ".qkv", 3, QKV + (int64_t)f0 * 3 * D, 3 * D, t3, pre + ".kvc", cross ? 2 : 0,
               KVC + (int64_t)f0 * 2 * D, 2 * D, t2, pre + ".ln_self_attn"));
  }
  {
    Timed tm(h, VAP_K_ATTN, st);
    AttnArgs a{QKV, 3 * D, t3, QKV + D, 3 * D, t3, QKV + 2 * D, 3 * D, t3, ATT, D, t1, h->P(pre + ".mha.m"), S, f1, H,
               0, scale};
    a.q0 = f0;
    HIPCHK(launch_attention<T>(a, st));
  }
  if (cross) {
    {
      Timed tm(h, VAP_K_TR_GEMM, st);  // out-proj + residual + LN_src + cross Q
      HIPCHK(lnp(ATT + (int64_t)f0 * D, pre + ".o", pre + ".qc", 1, QC + (int64_t)f0 * D, D, t1, "", 0, nullptr, 0, 0,
                 pre + ".ln_src_attn"));
    }
    {
      Timed tm(h, VAP_K_ATTN, st);
      AttnArgs a{QC, D, t1, KVC, 2 * D, t2, KVC + D, 2 * D, t2, ATT, D, t1, h->P(pre + ".mha_cross.m"), S, f1, H, 1,
                 scale};
      a.q0 = f0;
      HIPCHK(launch_attention<T>(a, st));
    }
  }
  {
    Timed tm(h, VAP_K_TR_GEMM, st);  // out-proj + residual + LN + FFN + residual (k_block.hip)
    BlockArgs b{Xf, ATT + (int64_t)f0 * D, S * nf, nf, t1, t1, h->W<T>(pre + (cross ? ".oc@rp" : ".o@rp")),
                h->W<T>(pre + ".w1@rp"), h->W<T>(pre + ".w2@rp"), h->P(pre + ".ln_ffnetwork.weight"),
                h->P(pre + ".ln_ffnetwork.bias"), 1e-5f};
    b.xb = xb_out ? xb_out + (int64_t)f0 * D : nullptr;
    if (!next.empty()) {  // + the next layer's LN_self . QKV (and raw-row cross K/V) from the same rows
      b.Wp = h->W<T>(next + (ncross ? ".qkvkvc@rp" : ".qkv@rp"));
      b.cp = (T*)(ws + p.QKVL) + (int64_t)(li + 1) * p.S * t3 + (int64_t)s0 * t3 + (int64_t)f0 * 3 * D;
      b.cr = ncross ? (T*)(ws + p.KVCL) + (int64_t)(cross ? ci + 1 : 0) * p.S * t2 + (int64_t)s0 * t2 + (int64_t)f0 * 2 * D
                    : nullptr;
      b.gamma2 = h->P(next + ".ln_self_attn.weight");
      b.beta2 = h->P(next + ".ln_self_attn.bias");
      b.np = 3;
      b.nr = ncross ? 2 : 0;
    }
    HIPCHK(launch_block(b, 0, st));
  }
  return VAP_OK;
}

// compute units of the current device (persistent kernels size their grid to the CUs they may use)
static int device_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// A persistent recurrence launch spins (bounded) on ready flags that kernels of the caller's stream
// publish.  Each of its workgroups fills a whole CU (W_hh resident: 160 KB LDS + every register),
// so the launch may take at most this many CUs, or the producers could find no CU to run on and
// every flag wait would time out.  Above it the forward uses plain per-range recurrence launches,
// which wait for nothing (the workgroups just queue).
static int lstm_wg_cap(const vap_handle* h) {
  return h->lstm_max_wg > 0 ? h->lstm_max_wg : std::max(1, device_cus() / 2);
}
// workgroups of one bf16 recurrence launch over S sequences (each publishes done counters)
static int rec_workgroups(const vap_handle*, int S) { return lstm_pair_workgroups(S); }
// groups of 16 sequences one persistent launch may take (at least one, whatever the cap)
static int rec_group_cap(const vap_handle* h) { return std::max(1, lstm_wg_cap(h) / 2); }
static bool persistent_fits(const vap_handle* h, int S) { return (S + 15) / 16 <= rec_group_cap(h); }
// workgroups of a persistent conv launch: the CUs the recurrence running beside it leaves free
static int conv_grid_cap(const vap_handle* h, int S) {
  return device_cus() - std::min(rec_workgroups(h, S), lstm_wg_cap(h));
}

// The bf16 recurrence of S sequences (gate rows: the pair-layout buffer GX from sequence seq0, h rows to
// out) on the pair-split kernel.  xg0 offsets the launch's slots in the exchange buffer (launches that
// may run concurrently use disjoint slots).
int launch_rec(vap_handle* h, const bf16* GX, int seq0, int S, int L4, int layer, bf16* out, int64_t out_stride,
               hipStream_t st, const LstmSync* sy, int xg0) {
  const std::string s = "_l" + std::to_string(layer);
  const size_t slot = lstm_pair_xbuf_bytes(16);
  const size_t need = (size_t)xg0 * slot + lstm_pair_xbuf_bytes(S);
  if (need > h->xbuf_bytes) {  // grow (rare): nothing may still use the old buffer
    HIPCHK(hipDeviceSynchronize());
    if (h->xbuf) HIPCHK(hipFree(h->xbuf));
    h->xbuf = nullptr;
    h->xbuf_bytes = 0;
    const size_t bytes = std::max(need, (size_t)64 * slot);
    HIPCHK(hipMalloc(&h->xbuf, bytes));
    HIPCHK(hipMemset(h->xbuf, 0, bytes));  // tags are >= 1: zero never matches
    // (hipMemset runs on the null stream, which the non-blocking side streams do not wait for)
    HIPCHK(hipDeviceSynchronize());
    h->xbuf_bytes = bytes;
  }
  const uint64_t span = (uint64_t)L4 + 1;
  if ((uint64_t)h->xtag + span + 1 > 0xFFFFFFFFull) {  // tag space exhausted (~4e9 steps): restart at 1
    HIPCHK(hipDeviceSynchronize());                    // no launch may still read the old tags
    HIPCHK(hipMemset(h->xbuf, 0, h->xbuf_bytes));
    HIPCHK(hipDeviceSynchronize());  // cleared before the launch on a non-blocking side stream reads it
    h->xtag = 0;
  }
  const unsigned tag0 = h->xtag + 1;  // this launch: tags tag0 .. tag0 + L4
  h->xtag += (unsigned)span;
  HIPCHK(launch_lstm_pair(GX, seq0, S, L4, h->W<bf16>("whh_pair" + s), out, out_stride, st, sy,
                          (unsigned char*)h->xbuf + (size_t)xg0 * slot, tag0, h->lstm_xplain));
  return VAP_OK;
}

// The fp32 recurrence of S sequences on the quad-split kernel (gate rows GX [S][L4][1024] fp32, h rows to
// out).  Shares the handle's exchange buffer and tag counter with the bf16 pair kernel (a handle runs one
// precision); xg0 offsets the launch's slots (launches that may run concurrently use disjoint slots).
int launch_rec_f32(vap_handle* h, const float* GX, int S, int L4, int layer, float* out, int64_t out_stride,
                   hipStream_t st, int xg0) {
  const std::string s = "_l" + std::to_string(layer);
  const size_t slot = lstm_quad_xbuf_bytes(16);
  const size_t need = (size_t)xg0 * slot + lstm_quad_xbuf_bytes(S);
  if (need > h->xbuf_bytes) {  // grow (rare): no launch may still use the old buffer
    HIPCHK(hipDeviceSynchronize());
    if (h->xbuf) HIPCHK(hipFree(h->xbuf));
    h->xbuf = nullptr;
    h->xbuf_bytes = 0;
    const size_t bytes = std::max(need, (size_t)8 * slot);
    HIPCHK(hipMalloc(&h->xbuf, bytes));
    HIPCHK(hipMemset(h->xbuf, 0, bytes));  // tags are >= 1: zero never matches
    HIPCHK(hipDeviceSynchronize());
    h->xbuf_bytes = bytes;
  }
  const uint64_t span = (uint64_t)L4 + 1;
  if ((uint64_t)h->xtag + span + 1 > 0xFFFFFFFFull) {  // tag space exhausted: restart at 1
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemset(h->xbuf, 0, h->xbuf_bytes));
    HIPCHK(hipDeviceSynchronize());
    h->xtag = 0;
  }
  const unsigned tag0 = h->xtag + 1;
  h->xtag += (unsigned)span;
  HIPCHK(launch_lstm_quad(GX, S, L4, h->W<bf16>("whhq" + s), out, out_stride, st,
                          (unsigned char*)h->xbuf + (size_t)xg0 * slot, tag0, h->err_dev));
  return VAP_OK;
}

// VapGPT.forward pipelined ALONG TIME (bf16, 1-layer LSTM).  The frames are cut into `nch` chunks;
// on the caller's stream the front end of chunk c computes only the conv / gate-projection rows
// that chunk needs (receptive fields: conv4 rows [., e) need conv3 rows < 2e+1, and so on down to
// conv1), then publishes ready[c]; one persistent LSTM launch on a side stream runs every
// sequence's recurrence, waiting at each chunk boundary and publishing done[c]; the back end of
// chunk c (downsample, every transformer layer on the chunk's frames -- causal, so only earlier
// keys are needed) waits for done[c].  The serial LSTM thus overlaps the whole front end and the
// earlier chunks' back ends, for all clips at once.
// Time-chunk schedule of a plan: frame chunks [fb[c], fb[c+1]) and the LSTM step at which each ends.
struct TcSched {
  int nch = 1;                          // recurrence chunks (ready / done hand-offs)
  int fb[vap_handle::MAXMB + 1]{};      // their frame boundaries
  int seq_end[vap_handle::MAXMB]{};     // LSTM step (conv4 row) at which each ends
  bool fe_pub[vap_handle::MAXMB]{};     // the front end publishes after chunk c (else it runs on)
  int nbe = 1;                          // back-end chunks: chunk k covers recurrence chunks
  int be_end[vap_handle::MAXMB + 1]{};  // [be_end[k-1], be_end[k]) (be_end[-1] = 0)
};
// Even chunks (the fallback of tc_schedule_split for short clips or custom chunk counts).
TcSched tc_schedule(const vap_handle* h, const Plan& p) {
  TcSched t;
  const int T_ = p.T;
  t.nch = std::min(h->time_chunks, vap_handle::MAXMB);
  t.nch = std::max(1, std::min(t.nch, T_ / 32));  // chunks of at least 32 frames
  const std::vector<double> wt(t.nch, 1.0);
  double tot = 0;
  for (double v : wt) tot += v;
  double acc = 0;
  t.fb[0] = 0;
  for (int c = 0; c < t.nch; ++c) {
    acc += wt[c];
    t.fb[c + 1] = c + 1 == t.nch ? T_ : std::max(t.fb[c] + 1, std::min(T_ - (t.nch - c - 1), (int)(T_ * acc / tot + 0.5)));
  }
  for (int c = 0; c < t.nch; ++c)
    t.seq_end[c] = c + 1 == t.nch ? (int)p.L[4] : std::min((int)p.L[4], 2 * t.fb[c + 1]);
  t.nbe = t.nch;
  for (int c = 0; c < t.nch; ++c) {
    t.fe_pub[c] = true;
    t.be_end[c] = c + 1;
  }
  return t;
}

// Forward schedule with separate front-end and back-end chunkings (h->tc_fe / h->tc_be: cumulative
// frame fractions of the boundaries, 1 excluded).  The step is bounded by the caller-stream work and
// by the chain "front end up to the first hand-off -> the whole recurrence -> back end after the last
// hand-off": the front end publishes in growing pieces (a short first one starts the recurrence early,
// each later one is ready before the recurrence gets there: the front end runs ~1.4x faster per
// frame than the recurrence), the back end works in shrinking pieces (a short last one after the
// recurrence ends).  The recurrence hands off at the union of both boundary sets.
TcSched tc_schedule_split(const vap_handle* h, const Plan& p) {
  const int T_ = p.T;
  if (h->tc_fe.empty() || h->tc_be.empty() || T_ < 128) return tc_schedule(h, p);
  std::vector<std::tuple<int, bool, bool>> bd;  // frame, front-end boundary, back-end boundary
  for (double f : h->tc_fe) bd.emplace_back((int)(T_ * f + 0.5), true, false);
  // long clips: a first front-end piece of the 20 s clip's first-piece size (120 frames), so the
  // recurrence starts as early as at 20 s (32 x 60 s: +1.5 %)
  if (h->tc_fe_auto && T_ > 1200) bd.emplace_back(120, true, false);
  if (h->tc_be_auto && T_ > 1200) {
    // long clips (the recurrence binds: 2 T dependent steps): chunks shrinking toward the end, so each
    // one's back end runs in the shadow of the recurrence's next chunk and the part after the
    // recurrence's end keeps its 20 s size: from the end ~360, 540, 810, ... frames (x1.5), the rest
    // one chunk, boundaries on 128 frames (whole attention q-blocks).  32 x 60 s: [1280, 2048, 2560];
    // 129.8k audio-s/s with the 20 s fraction 0.64, 142.2-143.6k with 0.4 / 0.7 / 0.88
    double sz = 360, pos = T_;
    int prev = T_;
    while ((pos -= sz) >= 384) {
      const int b = (int)pos / 128 * 128;
      if (b < prev) bd.emplace_back(b, false, true);
      prev = b;
      sz *= 1.5;
    }
  } else {
    for (double f : h->tc_be) bd.emplace_back((int)(T_ * f + 0.5), false, true);
  }
  std::sort(bd.begin(), bd.end());
  std::vector<std::tuple<int, bool, bool>> m;  // merged: boundaries closer than 24 frames become one
  for (auto& b : bd) {
    int f = std::get<0>(b);
    if (f < 24 || f > T_ - 24) continue;
    if (!m.empty() && f - std::get<0>(m.back()) < 24) {
      std::get<0>(m.back()) = f;
      std::get<1>(m.back()) = std::get<1>(m.back()) || std::get<1>(b);
      std::get<2>(m.back()) = std::get<2>(m.back()) || std::get<2>(b);
    } else {
      m.push_back(b);
    }
  }
  m.emplace_back(T_, true, true);
  if ((int)m.size() > vap_handle::MAXMB) return tc_schedule(h, p);
  TcSched t;
  t.nch = (int)m.size();
  t.fb[0] = 0;
  t.nbe = 0;
  for (int c = 0; c < t.nch; ++c) {
    t.fb[c + 1] = std::get<0>(m[c]);
    t.fe_pub[c] = std::get<1>(m[c]);
    if (std::get<2>(m[c])) t.be_end[t.nbe++] = c + 1;
  }
  for (int c = 0; c < t.nch; ++c)
    t.seq_end[c] = c + 1 == t.nch ? (int)p.L[4] : std::min((int)p.L[4], 2 * t.fb[c + 1]);
  return t;
}

// The recurrence of the time-chunked forward: ONE persistent launch on a side stream covers every
// sequence, waiting at each chunk boundary for ready[c] and publishing done[c].
int tc_launch_lstm(vap_handle* h, const Plan& p, const TcSched& t, const bf16* GX, unsigned char* ws, LstmSync& sy,
                   hipStream_t st, int gx_off = 0) {
  sy = LstmSync{};
  sy.gx_off = gx_off;
  sy.ready = h->sync_mem;
  sy.done = h->sync_mem + vap_handle::MAXMB;
  sy.error = h->err_dev;
  sy.epoch = ++h->epoch;
  sy.nr = t.nch;
  sy.time_mode = 1;
  for (int c = 0; c < t.nch; ++c) sy.seq_end[c] = t.seq_end[c];
  hipStream_t side = h->side[0];
  hipEvent_t fork = h->next_fork_event();
  HIPCHK(hipEventRecord(fork, st));
  HIPCHK(hipStreamWaitEvent(side, fork, 0));
  {
    Timed tm(h, VAP_K_LSTM_REC, side);
    if (int rc = launch_rec(h, GX, 0, p.S, (int)p.L[4], 0, (bf16*)(ws + p.H0) + 4 * D, p.sh, side, &sy, 0)) return rc;
  }
  // the back ends wait for these counts: raise them only once the launch is in the queue (a failed
  // launch must not leave later forwards waiting for arrivals that never come)
  const int nwg = rec_workgroups(h, p.S);
  for (int c = 0; c < t.nch; ++c) h->done_expect[c] += nwg;
  return VAP_OK;
}

// Heads on frames [f0, f1) of every clip (stereo, time-chunked back end): combinator (two GEMMs with
// the shared LN + GELU epilogue, the second adding onto the first), vap_head, va_classifier -- all
// row-wise (modules.py:411-449, model.py:257-261), so each back-end chunk finishes its own heads and
// only the last chunk's remain after the recurrence.  RAW holds the bf16 copy of the final x that
// the last layer's block kernel wrote.
int heads_tc(vap_handle* h, const Plan& p, unsigned char* ws, int f0, int f1, float* logits, float* vadl,
             hipStream_t st, int c0 = 0, int nb = -1) {
  // clips [c0, c0 + nb) only (sequences 2 c0 ..)
  using T = bf16;
  const int T_ = p.T, nf = f1 - f0, B = nb < 0 ? p.B : nb;
  const int64_t t1 = (int64_t)T_ * D;
  float* X = (float*)(ws + p.X) + (int64_t)2 * c0 * t1;
  T* RAW = (T*)(ws + p.RAW) + (int64_t)2 * c0 * t1;
  logits += (int64_t)c0 * T_ * 256;
  vadl += (int64_t)c0 * T_ * 2;
  Timed tm(h, VAP_K_HEADS, st);
  const int64_t o = (int64_t)f0 * D;
  // heads_kernel on the frame range [f0, f0 + nf) of every clip
  HeadsArgs ha{(const bf16*)(RAW + o), t1, B * nf, nf, (const bf16*)h->W<T>("comb_a@rp"),
               (const bf16*)h->W<T>("comb_b@rp"), (const bf16*)h->W<T>("head@rp"), h->P("ar.combinator.ln.weight"),
               h->P("ar.combinator.ln.bias"), h->P("vap_head.bias"), logits, 1e-5f, h->P("va_classifier.weight"),
               h->P("va_classifier.bias"), vadl, T_, f0};
  ha.xf = X + o;
  HIPCHK(launch_heads(ha, st));
  return VAP_OK;
}

// Sequence groups of the time-chunked back end (1 or 2, see tc_back_end).  Two need: the front end on
// side[1] (its join event passed in), per-chunk heads, whole clips in each half, and no back-end class
// timed (vap_timing brackets one stream's launches).
static int be_split_ways(const vap_handle* h, const Plan& p, bool fe_on_side1) {
  if (h->be_split < 2 || !fe_on_side1 || !h->heads_chunked || h->dims.cross_layers <= 0 || p.B < 2)
    return 1;
  const int tc = h->timing_cls;
  if (tc == VAP_K_DOWNSAMPLE || tc == VAP_K_TR_GEMM || tc == VAP_K_ATTN || tc == VAP_K_HEADS) return 1;
  return std::min(std::min(h->be_split, 3), p.B);
}

// Back end of the time-chunked forward: per chunk, wait for the recurrence (done[c]), downsample,
// every transformer layer on the chunk's frames; then heads over all clips and the join.
// fe_join (optional): the front-end stream's completion, joined into st at the end only (the back end
// reads the recurrence's h rows, which the done[] hand-off orders; nothing the front end writes)
int tc_back_end(vap_handle* h, const Plan& p, const TcSched& t, const LstmSync& sy, unsigned char* ws, float* logits,
                float* vadl, hipStream_t st, const unsigned* kernel_expect = nullptr, bool join = true,
                hipEvent_t fe_join = nullptr) {
  using T = bf16;
  const int S = p.S, T_ = p.T;
  const int64_t t1 = (int64_t)T_ * D;
  T* Hf = (T*)(ws + p.H0);
  float* X = (float*)(ws + p.X);
  // later chunks' front ends; the LSTM hand-off orders them
  const hipStream_t bst = st;
  // be_split = 2 (sequence halves on two streams: the caller's and the front-end stream, which joins
  // once the last front-end piece is done): each launch's last partial round of workgroups, and the
  // attention (VALU / MFMA) beside the row kernels (HBM), share the chip with the other half's launches
  const int nsp = be_split_ways(h, p, fe_join != nullptr && !kernel_expect && bst == st);
  if (nsp > 2) {  // the third group's stream follows everything the caller stream has queued so far
    hipEvent_t fk = h->next_fork_event();
    HIPCHK(hipEventRecord(fk, st));
    HIPCHK(hipStreamWaitEvent(h->side[2], fk, 0));
  }
  // (the second group on side[2] at normal priority, after the front end's end, measured -2.5 %)
  int rc;
  for (int k = 0; k < t.nbe; ++k) {
    const int c = t.be_end[k] - 1;  // the last recurrence chunk of back-end chunk k
    const int f0 = t.fb[k ? t.be_end[k - 1] : 0], f1 = t.fb[c + 1];
   for (int g = 0; g < nsp; ++g) {
    // clip boundaries of the groups (be_frac: the caller stream's share of two groups)
    auto cb = [&](int k) {
      if (k <= 0) return 0;
      if (k >= nsp) return p.B;
      if (nsp == 2) return std::min(p.B - 1, std::max(1, (int)(p.B * h->be_frac + 0.5)));
      return p.B * k / nsp;
    };
    const int sq0 = 2 * cb(g), sq1 = 2 * cb(g + 1);
    const hipStream_t bs = g == 0 ? bst : h->side[g];
    if (kernel_expect)  // captured streaming push: the hand-off as a kernel (graph-capturable)
      HIPCHK(launch_wait_geq(sy.done + c, kernel_expect[c], sy.error, bs));
    else
      HIPCHK(hipStreamWaitValue32(bs, sy.done + c, h->done_expect[c], hipStreamWaitValueGte, 0xFFFFFFFFu));
    {  // downsample: CConv1d k5 s2 causal + LayerNorm + GELU (encoder_components.py:485-499)
      Timed tm(h, VAP_K_DOWNSAMPLE, bs);
      GemmArgs ga = gargs(Hf + (int64_t)sq0 * p.sh + (int64_t)f0 * 2 * D, 2 * D, p.sh, h->W<T>("down"), 5 * D, D,
                          h->P("encoder.downsample.1.bias"), f1 - f0, sq1 - sq0, X + (int64_t)sq0 * t1 + (int64_t)f0 * D, D, t1);
      ga.norm = 2;
      ga.act = 2;
      ga.gamma = h->P("encoder.downsample.2.ln.weight");
      ga.beta = h->P("encoder.downsample.2.ln.bias");
      HIPCHK(hgemm<T>(h, ga, bs, true));
    }
    // per-chunk heads need the final x as bf16 from the last layer's fused block kernel
    const bool hchunk = h->heads_chunked && h->dims.cross_layers > 0;
    // layer list (name, cross attention, cross-K/V slot); the last layer's block kernel also writes x as
    // bf16 (RAW): the combinator's input, so the heads need no separate fp32 -> bf16 pass over x
    const int nl = h->dims.channel_layers + h->dims.cross_layers;
    auto lname = [&](int i) {
      return i < h->dims.channel_layers ? "ar_channel.layers." + std::to_string(i)
                                        : "ar.layers." + std::to_string(i - h->dims.channel_layers);
    };
    for (int li = 0; li < nl; ++li) {
      const bool cr = li >= h->dims.channel_layers, last = li + 1 == nl;
      const int ci = cr ? li - h->dims.channel_layers : 0;
      bf16* xb = cr && last ? (bf16*)(ws + p.RAW) : nullptr;
      const bool fuse = h->block_fuse && !last;
      if ((rc = tr_layer_tc(h, p, ws, lname(li), cr, li, ci, f0, f1, bs, xb, h->block_fuse && li > 0,
                            fuse ? lname(li + 1) : std::string(), li + 1 >= h->dims.channel_layers, sq0, sq1 - sq0)))
        return rc;
    }
    if (hchunk && (rc = heads_tc(h, p, ws, f0, f1, logits, vadl, bs, sq0 / 2, (sq1 - sq0) / 2))) return rc;
   }
  }
  if (!(h->heads_chunked && h->dims.cross_layers > 0) && (rc = heads<T>(h, p, ws, Range{0, p.B}, logits, vadl, bst, true)))
    return rc;
  if (nsp > 1) {  // the second half ran on the front-end stream, after its last piece: that joins both
    fe_join = h->next_fork_event();
    HIPCHK(hipEventRecord(fe_join, h->side[1]));
  }
  if (nsp > 2) {
    hipEvent_t j2 = h->next_fork_event();
    HIPCHK(hipEventRecord(j2, h->side[2]));
    HIPCHK(hipStreamWaitEvent(st, j2, 0));
  }
  if (fe_join) HIPCHK(hipStreamWaitEvent(st, fe_join, 0));
  if (!join) return VAP_OK;  // (captured push: the caller joins outside the graph)
  HIPCHK(hipEventRecord(h->mb_ev[0], h->side[0]));  // join: the LSTM launch has fully retired
  HIPCHK(hipStreamWaitEvent(st, h->mb_ev[0], 0));
  return VAP_OK;
}


// bf16 CPC rows of conv4 range [a4, b4) of every sequence, with the conv1..conv3 rows they need
// (k4 s2 p1 layers: rows [a, b) need input rows [2a-1, 2b+1) clipped to the layer; conv1 rows come
// from the fused conv0->conv1 kernel straight from the waveform), then their LSTM gate projections.
// With st2, conv2..4 and the gate projections run on st2 after an event on st (the caller keeps
// st for the next piece's conv01).  done_lv (optional, in / out): rows [0, done_lv[i]) of conv(i+1)
// exist already (an earlier piece of the same forward), so they are neither recomputed nor rewritten
// while an earlier piece's conv2..4 may still read them.
int conv_rows(vap_handle* h, const Plan& p, const float* wav, int64_t N, unsigned char* ws, bf16* GX, int64_t a4,
              int64_t b4, hipStream_t st, int64_t gx_off = 0, hipStream_t st2 = nullptr, int64_t* done_lv = nullptr) {
  using T = bf16;
  const int S = p.S;
  const int64_t* L = p.L;
  const std::string g = "encoder.encoder.gEncoder";
  T* Xs[4] = {(T*)(ws + p.X1), (T*)(ws + p.X2), (T*)(ws + p.X3), (T*)(ws + p.X4)};
  const int64_t ss[4] = {p.s1, p.s2, p.s3, p.s4};
  int64_t a[4], b[4];
  a[3] = a4;
  b[3] = b4;
  for (int i = 2; i >= 0; --i) {
    a[i] = std::max<int64_t>(0, 2 * a[i + 1] - 1);
    b[i] = std::min(L[i + 1], 2 * b[i + 1] + 1);
  }
  if (done_lv) {
    for (int i = 0; i < 3; ++i) a[i] = std::max(a[i], done_lv[i]);
    // after the first piece, conv1..3 ranges are whole 256-row tiles from where the last piece
    // stopped: the rows past what this piece needs are pulled forward from the next piece, not
    // extra work, and only the first and the last piece launch a partial tile per sequence
    for (int i = 2; i >= 0; --i) {
      if (a4 > 0) {
        const int64_t need = std::min(L[i + 1], 2 * b[i + 1] + 1);
        b[i] = std::min(L[i + 1], std::max(need, a[i] + (need - a[i] + 255) / 256 * 256));
      }
      b[i] = std::max(b[i], a[i]);
    }
  }
  if (a[0] < b[0]) {
    Timed tm(h, VAP_K_CONV1, st);
    HIPCHK(launch_conv01(wav, S, N, (int)L[0], (int)L[1], (const bf16*)h->W<T>("conv0_op"), h->fpacked.at("conv0_stat"),
                         h->P(g + ".batchNorm0.bias"), (const bf16*)h->W<T>("conv1"), (const bf16*)h->W<T>("conv1_ks"), h->P(g + ".conv1.bias"),
                         h->P(g + ".batchNorm1.weight"), h->P(g + ".batchNorm1.bias"), (bf16*)(Xs[0] + D), p.s1, st,
                         (int)a[0], (int)b[0], device_cus() - (p.S + 15) / 16));  // the recurrence holds a CU per 16 sequences
  }
  if (done_lv)
    for (int i = 0; i < 3; ++i) done_lv[i] = b[i];
  if (st2) {
    hipEvent_t fk = h->next_fork_event();
    HIPCHK(hipEventRecord(fk, st));
    HIPCHK(hipStreamWaitEvent(st2, fk, 0));
    st = st2;
  }

  for (int i = 1; i < 4; ++i) {  // conv2..4 (encoder_components.py:100-103)
    const std::string cs = std::to_string(i + 1);
    if (a[i] >= b[i]) continue;
    Timed tm(h, VAP_K_CONV234, st);
    ConvK4Args ca{Xs[i - 1] + a[i] * 2 * D, ss[i - 1], (int)(ss[i - 1] / D - 2 * a[i]), (const bf16*)h->W<T>("conv" + cs + "_ks"),
                  h->P(g + ".conv" + cs + ".bias"), h->P(g + ".batchNorm" + cs + ".weight"),
                  h->P(g + ".batchNorm" + cs + ".bias"), Xs[i] + D + a[i] * D, ss[i], (int)(b[i] - a[i])};
    ca.grid_cap = conv_grid_cap(h, S);
    HIPCHK(launch_convk4(ca, S, st));
  }
  // gate projections of rows [a4, b4) into ring slots (r + gx_off) mod L4: at most two pieces
  Timed tm(h, VAP_K_LSTM_PROJ, st);
  for (int64_t r = a4; r < b4;) {
    const int64_t slot = (r + gx_off) % L[4];
    const int64_t n = std::min(b4 - r, L[4] - slot);
    GemmArgs ga = gargs(Xs[3] + D + r * D, D, p.s4, h->W<T>("wih_l0"), D, 4 * D, h->fpacked.at("bias_l0"), (int)n, S,
                        GX, 4 * D, L[4] * 4 * D);
    ga.c_pair = 1;  // the pair-recurrence layout, ring slots slot .. slot + n - 1
    ga.c_t0 = (int)slot;
    ga.c_tn = (int)L[4];
    HIPCHK(hgemm<T>(h, ga, st, false));
    r += n;
  }
  return VAP_OK;
}

// VapGPT.forward pipelined ALONG TIME (bf16, 1-layer LSTM).  The frames are cut into `nch` chunks;
// on the caller's stream the front end of chunk c computes only the conv / gate-projection rows
// that chunk needs (receptive fields: conv4 rows [., e) need conv3 rows < 2e+1, and so on down to
// conv1), then publishes ready[c]; one persistent LSTM launch on a side stream runs every
// sequence's recurrence, waiting at each chunk boundary and publishing done[c]; the back end of
// chunk c (downsample, every transformer layer on the chunk's frames -- causal, so only earlier
// keys are needed) waits for done[c].  The serial LSTM thus overlaps the whole front end and the
// earlier chunks' back ends, for all clips at once.
int run_forward_tc(vap_handle* h, const Plan& p, const float* wav, int64_t N, float* logits, float* vadl,
                   unsigned char* ws, hipStream_t st) {
  using T = bf16;
  const TcSched t = tc_schedule_split(h, p);
  T* GX = (T*)(ws + p.GX);
  LstmSync sy;
  int rc;
  if ((rc = tc_launch_lstm(h, p, t, GX, ws, sy, st))) return rc;
  int64_t done_rows = 0, done_lv[3] = {0, 0, 0};
  int published = 0;
  // conv2..4 + gate projections (and the ready flags) on the front-end stream, conv01 on st
  // (timing mode, vap_timing, for a class that would run on the front-end stream: one stream, so its
  // events bracket only its own kernels; the bench times conv1, whose launches stay on st)
  const bool fe_timed = h->timing_serial || h->timing_cls == VAP_K_CONV234 || h->timing_cls == VAP_K_LSTM_PROJ;
  hipStream_t fst = h->fe_streams < 2 || fe_timed ? nullptr : h->side[1];
  for (int c = 0; c < t.nch; ++c) {  // front end, piece by piece (a piece ends at a front-end boundary)
    if (!t.fe_pub[c]) continue;
    if ((rc = conv_rows(h, p, wav, N, ws, GX, done_rows, t.seq_end[c], st, 0, fst, done_lv))) return rc;

    done_rows = t.seq_end[c];
    for (; published <= c; ++published)
      if (published != h->test_drop_ready)
        HIPCHK(hipStreamWriteValue32(fst ? fst : st, (void*)(sy.ready + published), sy.epoch, 0));
  }
  // join: anything after the forward on st follows the whole front end.  The back end itself waits
  // only for the recurrence (done[] flags), so its first chunk may start while the front-end stream
  // still runs the last piece's conv2..4 and gate projections
  hipEvent_t jn = nullptr;
  if (fst) {
    jn = h->next_fork_event();
    HIPCHK(hipEventRecord(jn, fst));
  }
  return tc_back_end(h, p, t, sy, ws, logits, vadl, st, nullptr, true, jn);
}

// VapGPT.forward (model.py:249-268).  Micro-batch pipeline: the batch is split into up to
// `microbatches` clip ranges; each range's front end runs on the caller's stream, its LSTM
// recurrence (a few CUs, serial over time) on a side stream, and its back end on the caller's
// stream after an event -- so the recurrences overlap the convolutions of later ranges and the
// transformer of earlier ones.  Every range writes disjoint workspace / output rows.
template <typename T>
int run_forward(vap_handle* h, const float* wav, int B, int64_t N, float* logits, float* vadl, unsigned char* ws,
                hipStream_t st, float* enc_out = nullptr) {
  const Plan p = plan_for(h, B, N);
  const int S = p.S;
  const int64_t* L = p.L;
  if constexpr (sizeof(T) == 2) {
    // A batch whose recurrence would not fit the persistent launch's CU budget runs the same
    // time-pipelined schedule slice by slice (identical kernels, so identical outputs per clip).
    if (h->use_time_chunks() && !enc_out && p.QKVL && !h->amap_active() && !persistent_fits(h, S)) {
      int rc;
      if ((rc = h->ensure_streams())) return rc;
      if (h->wait_value) {
        const int per = std::max(1, rec_group_cap(h) * 16 / 2);  // clips per slice (2 sequences each)
        const int ns = (B + per - 1) / per;
        for (int i = 0; i < ns; ++i) {
          const int c0 = (int)((int64_t)B * i / ns), c1 = (int)((int64_t)B * (i + 1) / ns);
          if ((rc = run_forward<T>(h, wav + (int64_t)c0 * 2 * N, c1 - c0, N, logits + (int64_t)c0 * p.T * 256,
                                   vadl + (int64_t)c0 * p.T * 2, ws, st)))
            return rc;
        }
        return VAP_OK;
      }
    }
  }
  // pad rows (conv zero padding lives in explicit rows), every region in one launch
  {
    constexpr int64_t R = D * (int64_t)sizeof(T);  // bytes per row
    ZeroRegions z;
    if constexpr (sizeof(T) == 4) {  // bf16 mode never materialises conv0
      T* X0 = (T*)(ws + p.X0);
      z.add(X0, p.s0 * sizeof(T), 2 * R);
      z.add(X0 + (L[0] + 2) * D, p.s0 * sizeof(T), 2 * R);
    }
    T* Xz[4] = {(T*)(ws + p.X1), (T*)(ws + p.X2), (T*)(ws + p.X3), (T*)(ws + p.X4)};
    const int64_t sz[4] = {p.s1, p.s2, p.s3, p.s4};
    for (int i = 0; i < 4; ++i) {
      z.add(Xz[i], sz[i] * sizeof(T), R);
      z.add(Xz[i] + (L[i + 1] + 1) * D, sz[i] * sizeof(T), R);
    }
    z.add(ws + p.H0, p.sh * sizeof(T), 4 * R);
    z.add(ws + p.H1, p.sh * sizeof(T), 4 * R);
    HIPCHK(launch_zero_regions(z, S, st));
  }

  const int NL = h->dims.lstm_layers;
  int m = h->microbatches < 1 ? 1 : h->microbatches;
  if (m > B) m = B;
  if (NL > 1 || h->amap_active() || h->dims.mono) m = 1;  // stacked LSTMs / attention maps / mono: serial
  // fp32: range i's recurrence launch goes to side stream i % NSIDE, so a range beyond NSIDE queued
  // behind an earlier range's whole recurrence (4 ranges: 90.6 ms of recurrence per forward against
  // 45.5 per launch); at most NSIDE ranges keep every recurrence on a stream of its own
  if constexpr (sizeof(T) == 4)
    if (m > vap_handle::NSIDE) m = vap_handle::NSIDE;
  std::vector<Range> rs;
  for (int i = 0; i < m; ++i) {
    const int c0 = (int)((int64_t)B * i / m), c1 = (int)((int64_t)B * (i + 1) / m);
    if (c1 > c0) rs.push_back({c0, c1 - c0, h->dims.mono ? 1 : 2});
  }
  int rc;
  if constexpr (sizeof(T) == 2) {
    if (h->use_time_chunks() && !enc_out && p.QKVL && !h->amap_active() && persistent_fits(h, S)) {
      if ((rc = h->ensure_streams())) return rc;
      if (h->wait_value) return run_forward_tc(h, p, wav, N, logits, vadl, ws, st);
    }
  }
  if (rs.size() == 1) {
    if ((rc = front_end<T>(h, p, wav, N, ws, rs[0], st))) return rc;
    for (int l = 0; l < NL; ++l)
      if ((rc = lstm_layer<T>(h, p, ws, l, rs[0], st, st))) return rc;
    return back_end<T>(h, p, ws, rs[0], logits, vadl, enc_out, st);
  }
  if ((rc = h->ensure_streams())) return rc;
  if constexpr (sizeof(T) == 2) {
    if (h->wait_value && persistent_fits(h, S)) {
      // One persistent LSTM launch on a side stream covers every range: its workgroups start as
      // each range's gate projection lands (ready flag written by this stream) and publish done
      // counters the back ends wait on.  No per-range launches, so no range queues behind another
      // range's recurrence on a shared side stream.
      const int nr = (int)rs.size();
      LstmSync sy{};
      sy.ready = h->sync_mem;
      sy.done = h->sync_mem + vap_handle::MAXMB;
      sy.error = h->err_dev;
      sy.epoch = ++h->epoch;
      sy.nr = nr;
      for (int i = 0; i < nr; ++i) sy.seq_end[i] = 2 * (rs[i].c0 + rs[i].nc);
      unsigned add[vap_handle::MAXMB] = {};
      const unsigned per_grp = 2u;  // workgroups per 16 sequences (pair split)
      for (int wg = 0; wg * 16 < S; ++wg) {  // done increments per range (16 sequences per group)
        const int s_first = wg * 16, s_last = std::min(S, s_first + 16) - 1;
        int ra = 0;
        while (sy.seq_end[ra] <= s_first) ++ra;
        int rb = ra;
        while (sy.seq_end[rb] <= s_last) ++rb;
        for (int r = ra; r <= rb; ++r) add[r] += per_grp;
      }
      hipStream_t side = h->side[0];
      hipEvent_t fork = h->next_fork_event();
      HIPCHK(hipEventRecord(fork, st));
      HIPCHK(hipStreamWaitEvent(side, fork, 0));
      {
        Timed tm(h, VAP_K_LSTM_REC, side);
        if ((rc = launch_rec(h, (const bf16*)(ws + p.GX), 0, S, (int)L[4], 0, (bf16*)((T*)(ws + p.H0) + 4 * D), p.sh,
                             side, &sy, 0)))
          return rc;
      }
      for (int i = 0; i < nr; ++i) h->done_expect[i] += add[i];  // only after a successful launch
      for (int i = 0; i < nr; ++i) {
        if ((rc = front_end<T>(h, p, wav, N, ws, rs[i], st))) return rc;
        if ((rc = lstm_layer<T>(h, p, ws, 0, rs[i], st, st, false))) return rc;
        HIPCHK(hipStreamWriteValue32(st, (void*)(sy.ready + i), sy.epoch, 0));
      }
      for (int i = 0; i < nr; ++i) {
        HIPCHK(hipStreamWaitValue32(st, sy.done + i, h->done_expect[i], hipStreamWaitValueGte, 0xFFFFFFFFu));
        if ((rc = back_end<T>(h, p, ws, rs[i], logits, vadl, enc_out, st))) return rc;
      }
      HIPCHK(hipEventRecord(h->mb_ev[0], side));  // join: the launch has fully retired
      HIPCHK(hipStreamWaitEvent(st, h->mb_ev[0], 0));
      return VAP_OK;
    }
  }
  int xg0 = 0;  // concurrent per-range recurrences use disjoint exchange slots
  for (size_t i = 0; i < rs.size(); ++i) {
    if ((rc = front_end<T>(h, p, wav, N, ws, rs[i], st))) return rc;
    hipStream_t side = h->side[i % vap_handle::NSIDE];
    if ((rc = lstm_layer<T>(h, p, ws, 0, rs[i], st, side, true, xg0))) return rc;
    xg0 += (rs[i].ns() + 15) / 16;
    HIPCHK(hipEventRecord(h->mb_ev[i], side));
  }
  for (size_t i = 0; i < rs.size(); ++i) {
    HIPCHK(hipStreamWaitEvent(st, h->mb_ev[i], 0));
    if ((rc = back_end<T>(h, p, ws, rs[i], logits, vadl, enc_out, st))) return rc;
  }
  return VAP_OK;
}


// ------------------------------------------------------------------------ streaming (C5)
// Conv4 row r of a window of n samples is CLEAN when no layer of its receptive field reaches a
// padding row or sample: k4 s2 p1 rows [lo, hi) need input rows [2lo-1, 2hi+1), conv1 (k8 s4 p2)
// [4lo-2, 4hi+2), conv0 (k10 s5 p3) samples [5lo-3, 5hi+2).  A clean row depends only on the samples
// under it, so after a hop of h = 160 k samples new row r equals old row r + k whenever both are
// clean (the conv stack is shift-equivariant with stride 160).
bool conv4_row_clean(const int64_t* L, int64_t n, int64_t r) {
  int64_t lo = r, hi = r + 1;
  for (int lvl = 3; lvl >= 1; --lvl) {  // conv4 -> conv3 -> conv2 -> conv1 input rows
    lo = 2 * lo - 1;
    hi = 2 * hi + 1;
    if (lo < 0 || hi > L[lvl]) return false;
  }
  lo = 4 * lo - 2;  // conv1 -> conv0 rows
  hi = 4 * hi + 2;
  if (lo < 0 || hi > L[0]) return false;
  lo = 5 * lo - 3;  // conv0 -> samples
  hi = 5 * hi + 2;
  return lo >= 0 && hi <= n;
}

}  // namespace

// Rolling-window stream (sds/run_sds.py:206-241 TurnTakingSDS.run: x.roll(-hop) + new samples at
// the end, model.probs(x) on the whole window; SURVEY config C5).  The window starts as zeros.  A
// push shifts the window by one hop; in bf16 mode the LSTM gate projections of the conv4 rows
// whose receptive field stays clean are carried over (shifted by hop/160 rows) and only the rows
// at the window edges -- the new audio plus the zero-padded first row -- run through the CPC conv
// stack.  The recurrence (zero state at the window start) and the transformer are recomputed, as
// in the reference, so the outputs equal a full forward of the window.
struct vap_stream {
  vap_handle* h = nullptr;
  int B = 0;
  int64_t W = 0, hop = 0;
  int hop_rows = 0;
  Plan p;
  unsigned char* ws = nullptr;
  float* win[2] = {};
  bf16* gx = nullptr;  // gate projections of the window: a ring, row r of the window in slot (r + gx_off) mod L4
  int64_t gx_off = 0;
  int cur = 0;
  int64_t pushes = 0;
  int64_t keep0 = 0, keep1 = 0;  // conv4 rows [keep0, keep1) carried over from the previous window
  bool reuse = false;
  // hipGraph-captured steady-state pushes (SURVEY config C5): the caller-stream part of a push (the
  // roll, the new rows' conv stack, the ready flags, the back end) is captured once per
  // (gate-ring offset, window buffer, output pointers) state -- the state repeats with period
  // L4 / gcd(L4, hop rows) pushes -- and replayed; the persistent recurrence launch stays eager on
  // the side stream, so the graph never depends on the runtime running its branches concurrently.
  bool graph = false;            // VAP_STREAM_GRAPH=0 disables
  float* hop_buf = nullptr;      // staging for the new hop (graph nodes read a fixed address)
  unsigned* gsync = nullptr;     // own ready[16] / done[16] / error, zeroed every push (epoch 1)
  struct GKey {
    int64_t off;
    int cur;
    const void* lg;
    const void* vd;
    bool operator<(const GKey& o) const {
      return std::tie(off, cur, lg, vd) < std::tie(o.off, o.cur, o.lg, o.vd);
    }
  };
  std::map<GKey, hipGraphExec_t> graphs;
  int64_t graph_replays = 0;
  hipStream_t cap = nullptr;  // capture stream (the caller's may be the legacy null stream, which cannot capture)
  ~vap_stream() {
    for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);
    if (cap) (void)hipStreamDestroy(cap);
    (void)hipFree(ws);
    for (int i = 0; i < 2; ++i) (void)hipFree(win[i]);
    (void)hipFree(gx);
    (void)hipFree(hop_buf);
    (void)hipFree(gsync);
  }
};

namespace {

// Caller-stream part of a steady-state push (captured into a hipGraph by stream_push_graph): roll the
// staged hop into window buffer nxt, the new rows' conv stack + gate projections with the ready
// flags as kernels, then the back end waiting on the recurrence's done counters with wait kernels.
int stream_main_graph(vap_stream* s, const TcSched& t, const LstmSync& sy, const unsigned* expect, int64_t off,
                      int nxt, float* logits, float* vadl, hipStream_t st) {
  vap_handle* h = s->h;
  const Plan& p = s->p;
  const int S = p.S;
  const int64_t W = s->W, hop = s->hop, L4 = p.L[4];
  HIPCHK(hipMemcpy2DAsync(s->win[nxt], W * sizeof(float), s->win[1 - nxt] + hop, W * sizeof(float),
                          (W - hop) * sizeof(float), S, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpy2DAsync(s->win[nxt] + (W - hop), W * sizeof(float), s->hop_buf, hop * sizeof(float),
                          hop * sizeof(float), S, hipMemcpyDeviceToDevice, st));
  const float* wav = s->win[nxt];
  int rc, published = 0;
  auto publish = [&](int64_t rows_ready) -> int {
    for (; published < t.nch && t.seq_end[published] <= rows_ready; ++published)
      if (published != h->test_drop_ready) HIPCHK(launch_flag_set((unsigned*)sy.ready + published, sy.epoch, st));
    return VAP_OK;
  };
  if (s->keep0 > 0 && (rc = conv_rows(h, p, wav, W, s->ws, s->gx, 0, s->keep0, st, off))) return rc;
  if ((rc = publish(s->keep1))) return rc;
  if ((rc = conv_rows(h, p, wav, W, s->ws, s->gx, s->keep1, L4, st, off))) return rc;
  if ((rc = publish(L4))) return rc;
  return tc_back_end(h, p, t, sy, s->ws, logits, vadl, st, expect, /*join=*/false);
}

int stream_push_graph(vap_stream* s, const float* hop_audio, float* logits, float* vadl, hipStream_t st) {
  vap_handle* h = s->h;
  const Plan& p = s->p;
  const int S = p.S;
  const int nxt = 1 - s->cur;
  const int64_t L4 = p.L[4];
  const int64_t off = (s->gx_off + s->hop_rows) % L4;
  const TcSched t = tc_schedule_split(h, p);
  // eager: stage the hop, zero the hand-off words, start the recurrence on the side stream
  HIPCHK(hipMemcpyAsync(s->hop_buf, hop_audio, (size_t)S * s->hop * sizeof(float), hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemsetAsync(s->gsync, 0, (2 * vap_handle::MAXMB + 1) * sizeof(unsigned), st));
  LstmSync sy{};
  sy.gx_off = (int)off;
  sy.ready = s->gsync;
  sy.done = s->gsync + vap_handle::MAXMB;
  sy.error = h->err_dev;
  sy.epoch = 1;
  sy.nr = t.nch;
  sy.time_mode = 1;
  for (int c = 0; c < t.nch; ++c) sy.seq_end[c] = t.seq_end[c];
  unsigned expect[vap_handle::MAXMB];
  for (int c = 0; c < t.nch; ++c) expect[c] = (unsigned)rec_workgroups(h, S);
  hipStream_t side = h->side[0];
  hipEvent_t fork = h->next_fork_event();
  HIPCHK(hipEventRecord(fork, st));
  HIPCHK(hipStreamWaitEvent(side, fork, 0));
  if (int rc = launch_rec(h, s->gx, 0, S, (int)L4, 0, (bf16*)(s->ws + p.H0) + 4 * D, p.sh, side, &sy, 0)) return rc;
  // captured: everything else on the caller's stream
  const vap_stream::GKey key{off, nxt, logits, vadl};
  auto it = s->graphs.find(key);
  if (it == s->graphs.end()) {
    if (s->graphs.size() >= 32) {  // a state cycle this long is not worth caching: run the part eagerly
      int rc = stream_main_graph(s, t, sy, expect, off, nxt, logits, vadl, st);
      if (rc) return rc;
    } else {
      HIPCHK(hipStreamBeginCapture(s->cap, hipStreamCaptureModeThreadLocal));
      const int rc = stream_main_graph(s, t, sy, expect, off, nxt, logits, vadl, s->cap);
      hipGraph_t g = nullptr;
      const hipError_t ec = hipStreamEndCapture(s->cap, &g);
      if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
      }
      if (ec != hipSuccess) return fail(VAP_ERR_HIP, std::string("stream capture: ") + hipGetErrorString(ec));
      hipGraphExec_t ex = nullptr;
      const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ei != hipSuccess) return fail(VAP_ERR_HIP, std::string("graph instantiate: ") + hipGetErrorString(ei));
      it = s->graphs.emplace(key, ex).first;
    }
  }
  if (it != s->graphs.end()) {
    HIPCHK(hipGraphLaunch(it->second, st));
    ++s->graph_replays;
  }
  HIPCHK(hipEventRecord(h->mb_ev[0], side));  // join: the recurrence launch has retired
  HIPCHK(hipStreamWaitEvent(st, h->mb_ev[0], 0));
  s->gx_off = off;
  s->cur = nxt;
  ++s->pushes;
  return VAP_OK;
}

int stream_push(vap_stream* s, const float* hop_audio, float* logits, float* vadl, hipStream_t st) {
  vap_handle* h = s->h;
  const Plan& p = s->p;
  const int S = p.S;
  const int nxt = 1 - s->cur;
  const int64_t W = s->W, hop = s->hop, L4 = p.L[4];
  if (s->graph && s->reuse && s->pushes > 0 && s->keep1 > s->keep0 && h->timing_cls == 0)
    return stream_push_graph(s, hop_audio, logits, vadl, st);
  // roll: window[:, :W-hop] = old window[:, hop:], window[:, W-hop:] = the new samples
  HIPCHK(hipMemcpy2DAsync(s->win[nxt], W * sizeof(float), s->win[s->cur] + hop, W * sizeof(float),
                          (W - hop) * sizeof(float), S, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpy2DAsync(s->win[nxt] + (W - hop), W * sizeof(float), hop_audio, hop * sizeof(float),
                          hop * sizeof(float), S, hipMemcpyDeviceToDevice, st));
  const float* wav = s->win[nxt];
  int rc;
  if (!s->reuse) {  // fp32 parity mode / no time-chunked path: full forward of the window
    rc = h->dims.precision == VAP_PRECISION_BF16 ? run_forward<bf16>(h, wav, s->B, W, logits, vadl, s->ws, st)
                                                 : run_forward<float>(h, wav, s->B, W, logits, vadl, s->ws, st);
    if (rc) return rc;
    s->cur = nxt;
    ++s->pushes;
    return VAP_OK;
  }
  bf16* GX = s->gx;
  // the window moved by hop_rows conv4 rows: carried rows keep their ring slots
  const int64_t off = s->pushes > 0 ? (s->gx_off + s->hop_rows) % L4 : 0;
  const TcSched t = tc_schedule_split(h, p);
  LstmSync sy;
  if ((rc = tc_launch_lstm(h, p, t, GX, s->ws, sy, st, (int)off))) return rc;
  int published = 0;
  auto publish = [&](int64_t rows_ready) -> int {  // ready[c] for every chunk whose steps are all available
    for (; published < t.nch && t.seq_end[published] <= rows_ready; ++published)
      if (published != h->test_drop_ready) HIPCHK(hipStreamWriteValue32(st, (void*)(sy.ready + published), sy.epoch, 0));
    return VAP_OK;
  };
  if (s->pushes > 0 && s->keep1 > s->keep0) {
    // carried-over gate projections (new row r = old row r + hop_rows) stay in their ring slots;
    // the recurrence starts on them (and the recomputed first row) while the new audio's rows go
    // through the conv stack
    if (s->keep0 > 0 && (rc = conv_rows(h, p, wav, W, s->ws, GX, 0, s->keep0, st, off))) return rc;
    if ((rc = publish(s->keep1))) return rc;
    if ((rc = conv_rows(h, p, wav, W, s->ws, GX, s->keep1, L4, st, off))) return rc;
  } else {
    int64_t done = 0;  // first push: the front end chunk by chunk, as run_forward_tc
    for (int c = 0; c < t.nch; ++c) {
      if ((rc = conv_rows(h, p, wav, W, s->ws, GX, done, t.seq_end[c], st, off))) return rc;
      done = t.seq_end[c];
      if ((rc = publish(done))) return rc;
    }
  }
  if ((rc = publish(L4))) return rc;
  if ((rc = tc_back_end(h, p, t, sy, s->ws, logits, vadl, st))) return rc;
  s->gx_off = off;
  s->cur = nxt;
  ++s->pushes;
  return VAP_OK;
}

int stream_zero(vap_stream* s, hipStream_t st) {
  const Plan& p = s->p;
  const int S = p.S;
  for (int i = 0; i < 2; ++i) HIPCHK(hipMemsetAsync(s->win[i], 0, (size_t)S * s->W * sizeof(float), st));
  s->cur = 0;
  s->pushes = 0;
  return VAP_OK;
}

}  // namespace


// A bounded hand-off wait of an earlier call on this handle timed out (its outputs are invalid):
// report it once and clear the word.  Reads host-mapped memory, no device sync.
static int take_handoff_error(vap_handle* h) {
  if (!h->err_host || __atomic_load_n(h->err_host, __ATOMIC_ACQUIRE) == 0) return VAP_OK;
  __atomic_store_n(h->err_host, 0u, __ATOMIC_RELEASE);
  return fail(VAP_ERR_HIP,
              "a persistent LSTM / stream hand-off wait timed out (~2 s) in an earlier call on this handle: "
              "that call's outputs are invalid");
}

// ============================================================================== C ABI
extern "C" {

const char* vap_last_error(void) { return g_err.c_str(); }

const char* vap_build_info(void) {
  return "libvap_hip gfx950 kernels: conv0-cn, mfma-gemm(implicit conv, row-norm epilogue), lstm-mfma, "
         "flash-attn-alibi, probs, labels";
}

int vap_create(const vap_dims* dims, vap_handle** out) {
  if (!dims || !out) return fail(VAP_ERR_INVALID, "null argument");
  if (dims->dim != D) return fail(VAP_ERR_UNSUPPORTED, "dim must be 256 (CPC encoder width)");
  if (dims->num_heads <= 0 || D % dims->num_heads || D / dims->num_heads != 64)
    return fail(VAP_ERR_UNSUPPORTED, "head_dim must be 64 (num_heads = 4)");
  if (dims->n_bins != 4) return fail(VAP_ERR_UNSUPPORTED, "n_bins must be 4 (256 VAP classes)");
  if (dims->lstm_layers < 1 || dims->channel_layers < 0 || dims->cross_layers < 0)
    return fail(VAP_ERR_INVALID, "bad layer counts");
  if (dims->precision != VAP_PRECISION_FP32 && dims->precision != VAP_PRECISION_BF16)
    return fail(VAP_ERR_INVALID, "bad precision");
  if (dims->mono != 0 && dims->mono != 1) return fail(VAP_ERR_INVALID, "bad mono flag");
  if (dims->va_history_bins < 0 || (!dims->mono && dims->va_history_bins))
    return fail(VAP_ERR_INVALID, "va_history_bins is a VapGPTMono option");
  vap_handle* h = new vap_handle();
  h->dims = *dims;
  if (const char* e = getenv("VAP_MICROBATCHES")) h->microbatches = atoi(e);
  if (const char* e = getenv("VAP_HEADS_CHUNKED")) h->heads_chunked = atoi(e) != 0;
  if (const char* e = getenv("VAP_TIME_CHUNKS")) h->time_chunks = atoi(e);
  if (const char* e = getenv("VAP_FE_STREAMS")) h->fe_streams = atoi(e);
  if (const char* e = getenv("VAP_LSTM_MAX_WG")) h->lstm_max_wg = atoi(e);
  if (const char* e = getenv("VAP_BLOCK_FUSE")) h->block_fuse = atoi(e) != 0;
  if (const char* e = getenv("VAP_BE_SPLIT")) h->be_split = atoi(e);
  if (const char* e = getenv("VAP_LSTM_XPLAIN")) h->lstm_xplain = atoi(e);
  if (const char* e = getenv("VAP_FP32_EXACT")) h->fp32_split = atoi(e) == 0;
  if (const char* e = getenv("VAP_FP32_QUAD")) h->fp32_quad = atoi(e) != 0;
  if (const char* e = getenv("VAP_BE_FRAC")) {  // the caller stream's share of two back-end groups, in (0, 1)
    const double f = atof(e);
    if (!(f > 0.0 && f < 1.0)) {
      delete h;
      return fail(VAP_ERR_INVALID, "VAP_BE_FRAC must be a number in (0, 1)");
    }
    h->be_frac = f;
  }
  auto parse_list = [](const char* e, std::vector<double>& out) {
    out.clear();
    std::string v = e;
    size_t a = 0;
    while (a < v.size()) {
      size_t b = v.find(',', a);
      if (b == std::string::npos) b = v.size();
      const double x = atof(v.substr(a, b - a).c_str());
      if (x > 0 && x < 1) out.push_back(x);
      a = b + 1;
    }
  };
  if (const char* e = getenv("VAP_TC_FE")) {
    parse_list(e, h->tc_fe);
    h->tc_fe_auto = false;
  }
  if (const char* e = getenv("VAP_TC_BE")) {
    parse_list(e, h->tc_be);
    h->tc_be_auto = false;
  }

  if (h->time_chunks > vap_handle::MAXMB) h->time_chunks = vap_handle::MAXMB;
  if (h->microbatches > vap_handle::MAXMB) h->microbatches = vap_handle::MAXMB;
  add_schema(h);
  // host-only: the schema (vap_num_params / vap_param_info) needs no device; each parameter's device
  // copy is allocated by its first vap_set_param
  *out = h;
  return VAP_OK;
}

void vap_destroy(vap_handle* h) { delete h; }

int vap_num_params(const vap_handle* h, int* n) {
  if (!h || !n) return fail(VAP_ERR_INVALID, "null argument");
  *n = (int)h->keys.size();
  return VAP_OK;
}

int vap_param_info(const vap_handle* h, int i, const char** key, int64_t* numel) {
  if (!h || i < 0 || i >= (int)h->keys.size()) return fail(VAP_ERR_INVALID, "param index out of range");
  if (key) *key = h->keys[i].c_str();
  if (numel) *numel = h->params.at(h->keys[i]).numel;
  return VAP_OK;
}

int vap_set_param(vap_handle* h, const char* key, const float* src, int64_t numel, void* stream) {
  if (!h || !key || !src) return fail(VAP_ERR_INVALID, "null argument");
  auto it = h->params.find(key);
  if (it == h->params.end()) return fail(VAP_ERR_WEIGHTS, std::string("unexpected key: ") + key);
  if (it->second.numel != numel)
    return fail(VAP_ERR_WEIGHTS, std::string("size mismatch for ") + key + ": expected " +
                                     std::to_string(it->second.numel) + " got " + std::to_string(numel));
  if (!it->second.dev) HIPCHK(hipMalloc(&it->second.dev, numel * sizeof(float)));
  HIPCHK(hipMemcpyAsync(it->second.dev, src, numel * sizeof(float), hipMemcpyDefault, (hipStream_t)stream));
  it->second.set = true;
  h->finalized = false;
  return VAP_OK;
}

int vap_finalize(vap_handle* h, void* stream) {
  if (!h) return fail(VAP_ERR_INVALID, "null handle");
  for (auto& k : h->keys)
    if (!h->params.at(k).set) return fail(VAP_ERR_WEIGHTS, "missing key: " + k);
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  for (auto& kv : h->packed) (void)hipFree(kv.second);
  for (auto& kv : h->fpacked) (void)hipFree(kv.second);
  h->packed.clear();
  h->fpacked.clear();
  h->packed_numel.clear();
  h->split_of.clear();
  const int rc = h->dims.precision == VAP_PRECISION_BF16 ? pack_all<bf16>(h, (hipStream_t)stream)
                                                          : pack_all<float>(h, (hipStream_t)stream);
  if (rc) return rc;
  const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) return fail(VAP_ERR_HIP, std::string("weight packing: ") + hipGetErrorString(e));
  h->finalized = true;
  return VAP_OK;
}

int vap_frame_lengths(int64_t n_samples, int64_t* lens) {
  if (!lens || n_samples <= 0) return fail(VAP_ERR_INVALID, "bad n_samples");
  frame_lengths(n_samples, lens);
  return VAP_OK;
}

int vap_workspace_size(const vap_handle* h, int batch, int64_t n_samples, size_t* bytes) {
  if (!h || !bytes || batch <= 0 || n_samples <= 0) return fail(VAP_ERR_INVALID, "bad argument");
  int64_t L[6];
  frame_lengths(n_samples, L);
  if (L[5] <= 0) return fail(VAP_ERR_INVALID, "waveform too short for one frame");
  *bytes = plan_for(h, batch, n_samples).total;
  return VAP_OK;
}

int vap_forward(vap_handle* h, const float* waveform, int batch, int64_t n_samples, float* logits, float* vad_logits,
                void* workspace, size_t workspace_bytes, void* stream) {
  if (!h || !waveform || !logits || !vad_logits || !workspace) return fail(VAP_ERR_INVALID, "null argument");
  if (h->dims.mono) return fail(VAP_ERR_INVALID, "mono handle: use vap_forward_mono");
  if (!h->finalized) return fail(VAP_ERR_WEIGHTS, "vap_finalize not called after loading parameters");
  if (batch <= 0 || n_samples <= 0) return fail(VAP_ERR_INVALID, "bad batch / n_samples");
  if (int rc = take_handoff_error(h)) return rc;
  size_t need = 0;
  int rc = vap_workspace_size(h, batch, n_samples, &need);
  if (rc) return rc;
  if (workspace_bytes < need) return fail(VAP_ERR_INVALID, "workspace too small: need " + std::to_string(need));
  return h->dims.precision == VAP_PRECISION_BF16
             ? run_forward<bf16>(h, waveform, batch, n_samples, logits, vad_logits, (unsigned char*)workspace,
                                 (hipStream_t)stream)
             : run_forward<float>(h, waveform, batch, n_samples, logits, vad_logits, (unsigned char*)workspace,
                                  (hipStream_t)stream);
}

int vap_forward_attention(vap_handle* h, const float* waveform, int batch, int64_t n_samples, float* logits,
                          float* vad_logits, float* self_attn, float* cross_attn, float* cross_self_attn,
                          void* workspace, size_t workspace_bytes, void* stream) {
  if (!h) return fail(VAP_ERR_INVALID, "null handle");
  h->amap[0] = self_attn;
  h->amap[1] = cross_attn;
  h->amap[2] = cross_self_attn;
  const int rc = vap_forward(h, waveform, batch, n_samples, logits, vad_logits, workspace, workspace_bytes, stream);
  h->amap[0] = h->amap[1] = h->amap[2] = nullptr;
  return rc;
}

int vap_forward_mono(vap_handle* h, const float* waveform, const float* va, const float* va_history, int batch,
                     int64_t n_samples, float* logits, void* workspace, size_t workspace_bytes, void* stream) {
  if (!h || !waveform || !va || !logits || !workspace) return fail(VAP_ERR_INVALID, "null argument");
  if (!h->dims.mono) return fail(VAP_ERR_INVALID, "vap_forward_mono needs a handle created with dims.mono = 1");
  if (!h->finalized) return fail(VAP_ERR_WEIGHTS, "vap_finalize not called after loading parameters");
  if (batch <= 0 || n_samples <= 0) return fail(VAP_ERR_INVALID, "bad batch / n_samples");
  if (int rc = take_handoff_error(h)) return rc;
  size_t need = 0;
  int rc = vap_workspace_size(h, batch, n_samples, &need);
  if (rc) return rc;
  if (workspace_bytes < need) return fail(VAP_ERR_INVALID, "workspace too small: need " + std::to_string(need));
  h->mono_va = va;
  h->mono_hist = va_history;
  rc = h->dims.precision == VAP_PRECISION_BF16
           ? run_forward<bf16>(h, waveform, batch, n_samples, logits, nullptr, (unsigned char*)workspace,
                               (hipStream_t)stream)
           : run_forward<float>(h, waveform, batch, n_samples, logits, nullptr, (unsigned char*)workspace,
                                (hipStream_t)stream);
  h->mono_va = h->mono_hist = nullptr;
  return rc;
}

int vap_encode_va(vap_handle* h, const float* va, const float* va_history, int rows, float* out, void* stream) {
  if (!h || !va || !out || rows <= 0) return fail(VAP_ERR_INVALID, "bad argument");
  if (!h->dims.mono) return fail(VAP_ERR_INVALID, "vap_encode_va needs a handle created with dims.mono = 1");
  if (!h->finalized) return fail(VAP_ERR_WEIGHTS, "vap_finalize not called after loading parameters");
  const int bins = h->dims.va_history_bins;
  const bool hist = bins > 0 && va_history;
  HIPCHK(hipMemsetAsync(out, 0, (size_t)rows * D * sizeof(float), (hipStream_t)stream));
  HIPCHK(launch_va_cond(out, va, hist ? va_history : nullptr, rows, bins, h->P("va_condition.weight"),
                        h->P("va_condition.bias"), hist ? h->P("va_cond_history.weight") : nullptr,
                        hist ? h->P("va_cond_history.bias") : nullptr, h->P("va_cond_ln.weight"),
                        h->P("va_cond_ln.bias"), (hipStream_t)stream));
  return VAP_OK;
}

int vap_stream_create(vap_handle* h, int batch, int64_t window_samples, int64_t hop_samples, void* stream,
                      vap_stream** out) {
  if (!h || !out) return fail(VAP_ERR_INVALID, "null argument");
  if (h->dims.mono) return fail(VAP_ERR_UNSUPPORTED, "streaming is a VapGPT (stereo) path");
  if (!h->finalized) return fail(VAP_ERR_WEIGHTS, "vap_finalize not called after loading parameters");
  if (batch <= 0 || window_samples <= 0 || hop_samples <= 0 || hop_samples > window_samples)
    return fail(VAP_ERR_INVALID, "bad batch / window / hop");
  int64_t L[6];
  frame_lengths(window_samples, L);
  if (L[5] <= 0) return fail(VAP_ERR_INVALID, "window too short for one frame");
  hipStream_t st = (hipStream_t)stream;
  auto* s = new vap_stream;
  s->h = h;
  s->B = batch;
  s->W = window_samples;
  s->hop = hop_samples;
  s->p = plan_for(h, batch, window_samples);
  const Plan& p = s->p;
  const int S = p.S;
  auto bail = [&](const char* what) {
    delete s;
    return fail(VAP_ERR_HIP, std::string("vap_stream_create: ") + what);
  };
  if (hipMalloc(&s->ws, p.total) != hipSuccess) return bail("workspace");
  for (int i = 0; i < 2; ++i)
    if (hipMalloc(&s->win[i], (size_t)S * window_samples * sizeof(float)) != hipSuccess) return bail("window");
  // carry-over is exact only for hops of whole conv4 rows (160 samples) on the time-chunked bf16 path
  const bool bf = h->dims.precision == VAP_PRECISION_BF16;
  if (bf && h->use_time_chunks() && h->ensure_streams()) return bail("streams");  // sets wait_value
  // (the carry-over push needs the persistent recurrence launch: within its CU cap)
  s->reuse = bf && h->use_time_chunks() && h->wait_value && hop_samples % 160 == 0 && persistent_fits(h, S);
  if (const char* e = getenv("VAP_STREAM_REUSE")) s->reuse = s->reuse && atoi(e) != 0;  // A/B: 0 = recompute
  if (s->reuse) {
    if (hipMalloc(&s->gx, (size_t)gx_pair_elems(S, L[4]) * sizeof(bf16)) != hipSuccess) return bail("gate buffer");
    s->hop_rows = (int)(hop_samples / 160);
    int64_t c0 = 0;
    while (c0 < L[4] && !conv4_row_clean(L, window_samples, c0)) ++c0;
    int64_t c1 = c0;
    while (c1 < L[4] && conv4_row_clean(L, window_samples, c1)) ++c1;
    s->keep0 = c0;
    s->keep1 = std::max(c0, c1 - s->hop_rows);  // new row r and old row r + hop_rows both clean
    // the persistent workspace's conv / LSTM pad rows are zero once and never written
    bf16* Xs[4] = {(bf16*)(s->ws + p.X1), (bf16*)(s->ws + p.X2), (bf16*)(s->ws + p.X3), (bf16*)(s->ws + p.X4)};
    const int64_t ss[4] = {p.s1, p.s2, p.s3, p.s4};
    for (int i = 0; i < 4; ++i) {
      if (launch_zero_rows<bf16>(Xs[i], S, ss[i], 1, st) != hipSuccess ||
          launch_zero_rows<bf16>(Xs[i] + (L[i + 1] + 1) * D, S, ss[i], 1, st) != hipSuccess)
        return bail("zero rows");
    }
    if (launch_zero_rows<bf16>((bf16*)(s->ws + p.H0), S, p.sh, 4, st) != hipSuccess) return bail("zero rows");
  }
  s->graph = s->reuse;
  if (const char* e = getenv("VAP_STREAM_GRAPH")) s->graph = s->graph && atoi(e) != 0;
  if (s->graph) {
    if (hipMalloc(&s->hop_buf, (size_t)S * hop_samples * sizeof(float)) != hipSuccess) return bail("hop staging");
    if (hipMalloc(&s->gsync, (2 * vap_handle::MAXMB + 1) * sizeof(unsigned)) != hipSuccess) return bail("sync words");
    if (hipStreamCreateWithFlags(&s->cap, hipStreamNonBlocking) != hipSuccess) return bail("capture stream");
  }
  if (stream_zero(s, st)) return bail("zero window");
  if (hipStreamSynchronize(st) != hipSuccess) return bail("sync");
  *out = s;
  return VAP_OK;
}

int vap_stream_push(vap_stream* s, const float* hop_audio, float* logits, float* vad_logits, void* stream) {
  if (!s || !hop_audio || !logits || !vad_logits) return fail(VAP_ERR_INVALID, "null argument");
  if (int rc = take_handoff_error(s->h)) return rc;
  return stream_push(s, hop_audio, logits, vad_logits, (hipStream_t)stream);
}

int vap_synchronize(vap_handle* h, void* stream) {
  if (!h) return fail(VAP_ERR_INVALID, "null handle");
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return take_handoff_error(h);
}

int vap_stream_info(const vap_stream* s, int* frames, int64_t* window_samples, int64_t* hop_samples,
                    int64_t* reused_rows, const float** window) {
  if (!s) return fail(VAP_ERR_INVALID, "null stream");
  if (frames) *frames = s->p.T;
  if (window_samples) *window_samples = s->W;
  if (hop_samples) *hop_samples = s->hop;
  if (reused_rows) *reused_rows = s->reuse ? s->keep1 - s->keep0 : 0;
  if (window) *window = s->win[s->cur];
  return VAP_OK;
}

int vap_stream_graphs(vap_stream* s, int* graphs, int64_t* replays, int* handoff_error) {
  if (!s) return fail(VAP_ERR_INVALID, "null stream");
  if (graphs) *graphs = (int)s->graphs.size();
  if (replays) *replays = s->graph_replays;
  if (handoff_error) {
    unsigned e = 0;
    if (s->h->err_host) {
      HIPCHK(hipDeviceSynchronize());
      e = __atomic_load_n(s->h->err_host, __ATOMIC_ACQUIRE);
    }
    *handoff_error = (int)e;
  }
  return VAP_OK;
}

int vap_stream_reset(vap_stream* s, void* stream) {
  if (!s) return fail(VAP_ERR_INVALID, "null stream");
  return stream_zero(s, (hipStream_t)stream);
}

void vap_stream_destroy(vap_stream* s) { delete s; }

int vap_encode(vap_handle* h, const float* waveform, int batch, int64_t n_samples, float* out, void* workspace,
               size_t workspace_bytes, void* stream) {
  if (!h || !waveform || !out || !workspace) return fail(VAP_ERR_INVALID, "null argument");
  if (!h->finalized) return fail(VAP_ERR_WEIGHTS, "vap_finalize not called after loading parameters");
  if (batch <= 0 || n_samples <= 0) return fail(VAP_ERR_INVALID, "bad batch / n_samples");
  if (int rc = take_handoff_error(h)) return rc;
  size_t need = 0;
  int rc = vap_workspace_size(h, batch, n_samples, &need);
  if (rc) return rc;
  if (workspace_bytes < need) return fail(VAP_ERR_INVALID, "workspace too small: need " + std::to_string(need));
  return h->dims.precision == VAP_PRECISION_BF16
             ? run_forward<bf16>(h, waveform, batch, n_samples, nullptr, nullptr, (unsigned char*)workspace,
                                 (hipStream_t)stream, out)
             : run_forward<float>(h, waveform, batch, n_samples, nullptr, nullptr, (unsigned char*)workspace,
                                  (hipStream_t)stream, out);
}

int vap_aggregate(const float* probs, int batch, int frames, int n_bins, int from_bin, int to_bin, float* out,
                  void* stream) {
  if (!probs || !out) return fail(VAP_ERR_INVALID, "null argument");
  if (n_bins != 4) return fail(VAP_ERR_UNSUPPORTED, "n_bins must be 4");
  if (from_bin < 0 || to_bin < from_bin || to_bin >= n_bins) return fail(VAP_ERR_INVALID, "bad bin limits");
  HIPCHK(launch_aggregate(probs, (int64_t)batch * frames, n_bins, from_bin, to_bin, out, (hipStream_t)stream));
  return VAP_OK;
}

int vap_vad_postprocess(const float* vad_logits, int batch, int frames, float cutoff, int max_fill_frames,
                        int max_omit_frames, float* out, void* stream) {
  if (!vad_logits || !out || batch <= 0 || frames <= 0) return fail(VAP_ERR_INVALID, "bad argument");
  HIPCHK(launch_vad_post(vad_logits, batch, frames, cutoff, max_fill_frames, max_omit_frames, out, (hipStream_t)stream));
  return VAP_OK;
}

int vap_probs(const float* logits, const float* vad_logits, int batch, int frames, int n_bins, int now0, int now1,
              int fut0, int fut1, float* probs, float* vad, float* p_now, float* p_future, float* H, void* stream) {
  if (!logits || !vad_logits || !probs || !vad || !p_now || !p_future || !H) return fail(VAP_ERR_INVALID, "null argument");
  if (n_bins != 4) return fail(VAP_ERR_UNSUPPORTED, "n_bins must be 4");
  if (now0 < 0 || now1 < now0 || now1 >= n_bins || fut0 < 0 || fut1 < fut0 || fut1 >= n_bins)
    return fail(VAP_ERR_INVALID, "bad bin limits");
  HIPCHK(launch_probs(logits, vad_logits, batch, frames, n_bins, now0, now1, fut0, fut1, probs, vad, p_now, p_future, H,
                      (hipStream_t)stream));
  return VAP_OK;
}

int vap_probs_loss(const float* logits, const float* vad_logits, int batch, int frames, int n_bins, int now0, int now1,
                   int fut0, int fut1, const int* bin_frames, float threshold, float* probs, float* vad, float* p_now,
                   float* p_future, float* H, int64_t* labels, float* loss, void* stream) {
  if (!logits || !vad_logits || !probs || !vad || !p_now || !p_future || !H || !bin_frames || !labels || !loss)
    return fail(VAP_ERR_INVALID, "null argument");
  if (n_bins != 4) return fail(VAP_ERR_UNSUPPORTED, "n_bins must be 4");
  if (now0 < 0 || now1 < now0 || now1 >= n_bins || fut0 < 0 || fut1 < fut0 || fut1 >= n_bins)
    return fail(VAP_ERR_INVALID, "bad bin limits");
  int horizon = 0;
  for (int i = 0; i < n_bins; ++i) horizon += bin_frames[i];
  if (frames - 1 < horizon)
    return fail(VAP_ERR_TOO_SHORT, "maximum size for tensor at dimension 1 is " + std::to_string(frames - 1) +
                                       " but size is " + std::to_string(horizon));
  if (horizon > 128) return fail(VAP_ERR_UNSUPPORTED, "projection horizon above 128 frames");
  HIPCHK(launch_probs_loss(logits, vad_logits, batch, frames, n_bins, now0, now1, fut0, fut1, bin_frames, threshold,
                           probs, vad, p_now, p_future, H, labels, loss, (hipStream_t)stream));
  return VAP_OK;
}

int vap_labels_loss(const float* logits, const float* va, int batch, int frames, const int* bin_frames, int n_bins,
                    float threshold, int64_t* labels, float* loss, void* stream) {
  if (!va || !bin_frames || !labels || (logits && !loss)) return fail(VAP_ERR_INVALID, "null argument");
  if (n_bins != 4) return fail(VAP_ERR_UNSUPPORTED, "n_bins must be 4");
  int horizon = 0;
  for (int i = 0; i < n_bins; ++i) horizon += bin_frames[i];
  if (frames - 1 < horizon)
    return fail(VAP_ERR_TOO_SHORT, "maximum size for tensor at dimension 1 is " + std::to_string(frames - 1) +
                                       " but size is " + std::to_string(horizon));
  HIPCHK(launch_labels_loss(logits, va, batch, frames, bin_frames, n_bins, threshold, labels, loss, (hipStream_t)stream));
  return VAP_OK;
}

int vap_test_plan(const vap_handle* h, int batch, int64_t n_samples, int64_t* out) {
  if (!h || !out || batch <= 0 || n_samples <= 0) return fail(VAP_ERR_INVALID, "bad argument");
  const Plan p = plan_for(h, batch, n_samples);
  const size_t v[] = {p.X1, p.X2, p.X3, p.X4, p.GX, p.H0, p.X, p.total};
  const int64_t st[] = {p.s1, p.s2, p.s3, p.s4, p.sh};
  for (int i = 0; i < 8; ++i) out[i] = (int64_t)v[i];
  for (int i = 0; i < 5; ++i) out[8 + i] = st[i];
  return VAP_OK;
}

int vap_test_xtag(vap_handle* h, int64_t set, int64_t* get) {
  if (!h) return fail(VAP_ERR_INVALID, "null handle");
  if (get) *get = (int64_t)h->xtag;
  if (set >= 0) {
    if (set > 0xFFFFFFFFll) return fail(VAP_ERR_INVALID, "tag out of range");
    h->xtag = (unsigned)set;
  }
  return VAP_OK;
}

int vap_test_drop_ready(vap_handle* h, int chunk) {
  if (!h) return fail(VAP_ERR_INVALID, "null handle");
  h->test_drop_ready = chunk < 0 ? -1 : chunk;
  return VAP_OK;
}

int vap_test_lstm_xplain(vap_handle* h, int policy) {
  if (!h) return fail(VAP_ERR_INVALID, "null handle");
  if (policy < -1 || policy > 1) return fail(VAP_ERR_INVALID, "policy must be -1, 0 or 1");
  h->lstm_xplain = policy;
  return VAP_OK;
}

int vap_timing(vap_handle* h, int cls) {
  if (!h) return fail(VAP_ERR_INVALID, "null handle");
  h->timing_serial = cls < 0;
  h->timing_cls = cls < 0 ? -cls : cls;
  h->ev_used = 0;
  return VAP_OK;
}

int vap_timing_read(vap_handle* h, double* total_ms, int* launches) {
  if (!h || !total_ms || !launches) return fail(VAP_ERR_INVALID, "null argument");
  double tot = 0.0;
  for (size_t i = 0; i < h->ev_used; ++i) {
    HIPCHK(hipEventSynchronize(h->ev[i].second));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, h->ev[i].first, h->ev[i].second));
    tot += ms;
  }
  *total_ms = tot;
  *launches = (int)h->ev_used;
  h->ev_used = 0;
  return VAP_OK;
}

}  // extern "C"
