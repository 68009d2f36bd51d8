// Internal launch interface between the engine (vap_engine.cpp) and the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct GemmArgs {
  const void* A;          // storage type T
  int64_t lda;            // row stride (elements); may be < K for implicit conv
  int64_t a_seq_stride;   // per-sequence stride (elements)
  const void* W;          // [N][K] storage type T
  int K, N;
  const float* bias;      // [N] or null
  int M_per_seq, n_seq;   // M = M_per_seq * n_seq
  void* C;                // TOut
  int64_t ldc, c_seq_stride;
  const float* add;       // fp32 addend (may alias C when TOut == float) or null
  int64_t ld_add, add_seq_stride;
  const float* gamma;     // norm affine (N == 256)
  const float* beta;
  float eps;
  int norm;               // 0 none, 1 ChannelNorm (unbiased var), 2 LayerNorm (biased var)
  int act;                // 0 none, 1 relu, 2 gelu(erf)
  // c_pair = 1 (bf16 LSTM gate projection, N = 1024, W rows in gx_wrow order): C is the gate buffer in the
  // pair-recurrence layout (gx_pair_block): a tile is 16 time steps x 16 sequences (of sequences
  // c_s0 + 16k ..), row t of sequence s lands in ring slot (c_t0 + t) mod c_tn; ldc / c_seq_stride unused
  int c_pair = 0, c_s0 = 0, c_t0 = 0, c_tn = 0;
  // small_tiles = 1: the 128-row register-staged kernel even for bf16 (more workgroups for short launches;
  // chosen by the caller per call site, never by M, so outputs stay batch-invariant)
  int small_tiles = 0;
  // split = 1 (fp32 operands, TOut float): W is the split weight [N][K/32][64] bf16 (launch_split_bf16) and the
  // product runs as three bf16 MFMAs per tile-step (k_gemm.hip gemm3_kernel), K % 32 == 0
  int split = 0;
};

template <typename T, typename TOut>
hipError_t launch_gemm(const GemmArgs& g, hipStream_t st);
// fp32 W [n / K][K] -> bf16 [n / K][K / 32][64]: per 32-k block hi = bf16(x) then lo = bf16(x - hi) (the split
// weight rows of gemm3_kernel)
hipError_t launch_split_bf16(const float* in, bf16* out, int64_t n, int K, hipStream_t st);

// bf16 CPC conv2..4 (k4 s2 p1, 256 -> 256) + bias + ChannelNorm + ReLU (k_conv234.hip).  `in` points at
// the buffer row 2*a of the first output row a of the range (one zero pad row in front of each
// sequence), in_rows = rows readable per sequence from there (>= 2M + 2); W in the k-step-major
// layout [tap*8 + cb][256][32] (launch_pack_kstep of the [N][tap*256 + ci] packing); out = row a.
struct ConvK4Args {
  const bf16* in;
  int64_t in_seq_stride;
  int in_rows;
  const bf16* W;
  const float* bias;
  const float* gamma;
  const float* beta;
  bf16* out;
  int64_t out_seq_stride;
  int M;
  int dbg = 0;  // diagnostics (tools/diag_convk4.py): 1 raw conv + bias out, 2 G := 1, 4 W := 1,
                // 16 phase stamps of workgroups (0..7, seq 0) into stamps[8][12]
  unsigned long long* stamps = nullptr;
  int grid_cap = 0;  // workgroups of the persistent launch (the CUs free beside the recurrence; 0: all)
};
hipError_t launch_convk4(const ConvK4Args& a, int S, hipStream_t st);
// bf16 256x256-tile LDS-DMA variant (k_gemm2.hip); launch_gemm<bf16, *> dispatches to it
template <typename TOut>
hipError_t launch_gemm2(const GemmArgs& g, hipStream_t st);

// conv0 (1 -> 256, k10 s5 p3) + ChannelNorm + ReLU, time-major output with pad rows; 2B sequences
// (stereo clips) or nseq when given (mono: one sequence per clip).
template <typename T>
hipError_t launch_conv0(const float* wav, int B, int64_t N, int L0, const float* w0, const float* b0,
                        const float* gamma, const float* beta, T* out, int64_t out_seq_stride, hipStream_t st,
                        int nseq = -1);
// graph-capturable stream hand-offs (streaming push): *p = v after the preceding work; wait until *p >= v
hipError_t launch_flag_set(unsigned* p, unsigned v, hipStream_t st);
hipError_t launch_wait_geq(const unsigned* p, unsigned v, unsigned* err, hipStream_t st);
// VapGPTMono VA conditioning (vap/model.py:317-323, 352-357): x[r] += LayerNorm(Wv va[r] + bv
// (+ Wh hist[r] + bh)) for each of `rows` 256-wide rows; va [rows][2], hist [rows][bins] or NULL.
hipError_t launch_va_cond(float* x, const float* va, const float* hist, int rows, int bins, const float* Wv,
                          const float* bv, const float* Wh, const float* bh, const float* gamma, const float* beta,
                          hipStream_t st);

// Zero `rows` rows of width 256 at `base + s*seq_stride` for every sequence (pad rows).
template <typename T>
hipError_t launch_zero_rows(T* base, int n_seq, int64_t seq_stride, int rows, hipStream_t st);
// several per-sequence byte ranges zeroed in ONE launch (the conv / LSTM pad rows of a forward)
struct ZeroRegion {
  void* base;
  int64_t seq_stride_bytes;
  int64_t bytes;  // per sequence, multiple of 16
};
struct ZeroRegions {
  static constexpr int MAX = 16;
  ZeroRegion r[MAX];
  int n = 0;
  void add(void* base, int64_t seq_stride_bytes, int64_t bytes) { r[n++] = ZeroRegion{base, seq_stride_bytes, bytes}; }
};
hipError_t launch_zero_regions(const ZeroRegions& z, int n_seq, hipStream_t st);

// LayerNorm over 256 (biased var) of fp32 rows -> T, optional raw fp32->T copy.
template <typename T>
hipError_t launch_layernorm(const float* x, int64_t rows, const float* gamma, const float* beta, float eps,
                            T* out, T* raw, hipStream_t st);

// LSTM recurrence.  gx: [S][T][4H] fp32 (x W_ih^T + b_ih + b_hh), whh_packed: fragment-ordered
// W_hh (storage T), out: T rows with stride out_seq_stride, h (256) per row.
template <typename T>
hipError_t launch_lstm(const float* gx, int S, int Tn, const T* whh_packed, T* out, int64_t out_seq_stride,
                       hipStream_t st);
template <typename T>
hipError_t launch_pack_whh(const float* whh, T* packed, hipStream_t st);
// bf16 perf mode: W_hh resident in VGPRs + LDS (8 waves / CU), gx in bf16 [S][T][1024]
// Cross-stream hand-off for a single persistent LSTM launch covering several clip ranges: a
// workgroup waits until ready[r] >= epoch for the ranges r its 16 sequences fall in (written by the
// producing stream after the range's input projection), and on completion adds 1 to done[r] for
// each of them (the consuming stream waits for its expected count).  ready == nullptr: no hand-off.
struct LstmSync {
  const unsigned* ready;
  unsigned* done;
  unsigned* error;   // set to 1 if a ready flag did not arrive within ~2 s (never expected)
  unsigned epoch;
  int nr;            // number of ranges
  int seq_end[16];   // exclusive end sequence of each range (time_mode: exclusive end STEP of each
                     // time chunk: every workgroup waits ready[c] before the chunk and adds 1 to
                     // done[c] after it)
  int time_mode;
  int gx_off = 0;    // gate rows form a ring: step t reads gx row (t + gx_off) mod Tn (streaming)
  unsigned xtag = 0;  // lstm_pair: exchange tags of this launch are xtag (XCC handshake) .. xtag + Tn (steps);
                      // strictly above every earlier launch's on the same exchange slots (set by launch_lstm_pair)
  int xplain = 0;       // lstm_pair: exchange stores with the default policy even across XCDs (experiment; the
                        // XCC-id handshake picks that policy by itself when both halves share an XCD)
  int stamp_t0 = 100;   // lstm_pair<ST>: first of the 4 stamped steps (VAP_LSTM_STAMP_T0)
  int handoff_trace = 0;  // lstm_pair (VAP_LSTM_HANDOFF=1): workgroup 0 records s_memrealtime around each hand-off
};
// diagnostics: [0] launch start, then per time chunk c: [1 + 3c] ready wait begins, [2 + 3c] ready seen,
// [3 + 3c] done published (s_memrealtime, 100 MHz) of the last lstm_pair launch with handoff_trace
hipError_t read_lstm_handoff(unsigned long long* out);
hipError_t read_lstm_xcc(unsigned* out);  // XCD handshake record of the last pair launch (64 blocks)
// prescaled: W_ih / W_hh / biases packed with the gate scales (launch_pack_wih_prescaled,
// launch_pack_whh_resident(.., true)): gates arrive as -log2e (i, f, o) / 2 log2e (g) multiples
hipError_t launch_lstm_resident(const bf16* gx, int S, int Tn, const bf16* whh_packed, bf16* out,
                                int64_t out_seq_stride, hipStream_t st, const LstmSync* sync, bool prescaled = false);
hipError_t launch_pack_whh_resident(const float* whh, bf16* packed, hipStream_t st, bool prescaled = false);
// W_hh split over a pair of workgroups (k_lstm.hip lstm_pair_kernel): pre-scaled packing, the
// exchange buffer it needs for S sequences (zeroed once; tags carry the launch epoch, which must
// differ between launches that share the buffer), and the workgroups one launch runs
// gx: the pair-layout gate buffer (gx_pair_block) whose sequence seq0 is this launch's sequence 0
hipError_t launch_lstm_pair(const bf16* gx, int seq0, int S, int Tn, const bf16* whh_pair, bf16* out, int64_t out_seq_stride,
                            hipStream_t st, const LstmSync* sync, void* xbuf, unsigned xtag,
                            int xplain = 0, int quad = 0);
hipError_t launch_pack_whh_pair(const float* whh, bf16* packed, hipStream_t st);
size_t lstm_pair_xbuf_bytes(int S);
// fp32 parity mode: W_hh split over a QUAD of workgroups (k_lstm.hip lstm_quad_kernel), split-bf16 products:
// gx fp32 [S][Tn][1024] (biases included), whh_quad from launch_pack_whh_quad ([4][4][64][64][8] bf16), h rows
// fp32 to out (row t of sequence s at out + s*out_seq_stride + t*256); xbuf: lstm_quad_xbuf_bytes(S), zeroed
// once; xtag >= 1: this launch's tags are xtag .. xtag + Tn - 1 (above every earlier launch's on the same slots)
hipError_t launch_lstm_quad(const float* gx, int S, int Tn, const bf16* whh_quad, float* out, int64_t out_seq_stride,
                            hipStream_t st, void* xbuf, unsigned xtag, unsigned* err);
hipError_t launch_pack_whh_quad(const float* whh, bf16* packed, hipStream_t st);
size_t lstm_quad_xbuf_bytes(int S);
// The bf16 LSTM gate buffer in the pair-recurrence layout (k_lstm.hip lstm_pair_kernel): for each group of
// 16 sequences, ring slot and 16-unit block ub = 8p + w (half p of the pair, wave w), one 2 KiB block of
// 2 halves x 64 lanes x 16 bytes, lane = 16 lg + s % 16 holding units 16ub + 4lg .. +3 of sequence s:
// half 0 = gates 0, 1 (4 bf16 each), half 1 = gates 2, 3.  A recurrence wave reads its step as two 1 KiB
// lines-aligned loads, and a gate-projection wave (16 steps x 16 sequences per tile) writes them alike.
// Element offset of the block:
__host__ __device__ inline int64_t gx_pair_block(int grp, int slot, int ub, int tn) {
  return (((int64_t)grp * tn + slot) * 16 + ub) * 1024;
}
// element of gate row (g, u) of sequence s, slot `slot`
__host__ __device__ inline int64_t gx_pair_off(int s, int slot, int g, int u, int tn) {
  return gx_pair_block(s >> 4, slot, u >> 4, tn) + (g >> 1) * 512 + (((u >> 2) & 3) * 16 + (s & 15)) * 8 + (g & 1) * 4 +
         (u & 3);
}
inline int64_t gx_pair_elems(int S, int64_t Tn) { return (int64_t)((S + 15) / 16) * 16 * Tn * 1024; }
// W_ih / bias row order of the gate projection in c_pair mode: output column n = 64ub + 16g + (u % 16), so
// a GEMM lane's 4 column blocks are the 4 gates of its 4 units (one full record)
__host__ __device__ inline int gx_wrow(int g, int u) { return (u >> 4) * 64 + g * 16 + (u & 15); }
// [S][Tn][1024] natural gate order -> the pair layout (kernel tests)
hipError_t launch_pack_gx_pair(const bf16* in, bf16* out, int S, int Tn, hipStream_t st);
// workgroups of one launch_lstm_pair launch (each publishes the done counters): 2 per 16 sequences, 4 with quad
// (lstm_quadb_kernel: the same packed W_hh, gate layout and exchange buffer)
int lstm_pair_workgroups(int S, int quad = 0);
hipError_t launch_scale_gates(const bf16* in, bf16* out, int64_t n, hipStream_t st);
hipError_t launch_pack_wih_prescaled(const float* wih, bf16* packed, const float* bih, const float* bhh, float* bias,
                                     hipStream_t st);

struct AttnArgs {
  const void* Q; int64_t q_ld, q_seq;     // head h at column h*64
  const void* K; int64_t k_ld, k_seq;
  const void* V; int64_t v_ld, v_seq;
  void* O; int64_t o_ld, o_seq;
  const float* slopes;                    // [H]
  int S, T, H;
  int kv_swap;                            // 0: self (K/V of s); 1: cross (K/V of s ^ 1, clip-major pairs)
  float scale;
  int q0 = 0;                             // queries [q0, T) against keys [0, T) (time-chunked back end;
                                          // bf16 attn3 only); Q / O still point at row 0
  int split = 0;                          // fp32: products on split-bf16 operands (k_attn.hip attn_split_kernel)
};
template <typename T>
hipError_t launch_attention(const AttnArgs& a, hipStream_t st);
// attention weights of one layer (attention=True): out[s * out_seq + h * out_head + i * T + j] fp32
template <typename T>
hipError_t launch_attn_probs(const AttnArgs& a, float* out, int64_t out_seq, int64_t out_head, hipStream_t st);

// va_classifier on both towers: vad[b][t][c] = dot(x[2b+c][t], w) + bias (x fp32, clip-major seqs)
hipError_t launch_vad_head(const float* x, int B, int Tn, const float* w, const float* bias, float* vad, hipStream_t st);
// frames [t0, t0 + nt) of every sequence: x points at frame t0 of sequence 0, sequences x_seq apart
hipError_t launch_vad_head_rows(const float* x, int64_t x_seq, int B, int Tn, int t0, int nt, const float* w,
                                const float* bias, float* vad, hipStream_t st);
// rows [0, rows) of n_seq sequences of 256-wide fp32 rows -> T (sequence strides in elements)
template <typename T>
hipError_t launch_convert_rows(const float* in, int64_t in_seq, T* out, int64_t out_seq, int n_seq, int rows,
                               hipStream_t st);

hipError_t launch_probs(const float* logits, const float* vad_logits, int B, int Tn, int n_bins, int now0, int now1,
                        int fut0, int fut1, float* probs, float* vad, float* p_now, float* p_future, float* H,
                        hipStream_t st);
// probs epilogue + labels + loss in two launches (labels from the VAD logits through LDS, the loss
// from the softmax's max / sum): what VapGPT.probs needs after the forward
hipError_t launch_probs_loss(const float* logits, const float* vad_logits, int B, int Tn, int n_bins, int now0,
                             int now1, int fut0, int fut1, const int* bin_frames, float threshold, float* probs,
                             float* vad, float* p_now, float* p_future, float* H, int64_t* labels, float* loss,
                             hipStream_t st);
hipError_t launch_labels_loss(const float* logits, const float* va, int B, int Tn, const int* bin_frames, int n_bins,
                              float threshold, int64_t* labels, float* loss, hipStream_t st);

// fp32 -> storage conversion (weights packing) and small helpers
template <typename T>
hipError_t launch_convert(const float* in, T* out, int64_t n, hipStream_t st);
// out[n][j*C + c] = in[n][c][j]  (conv weight (N, C, KW) -> K-contiguous (tap, channel) order)
template <typename T>
hipError_t launch_pack_conv(const float* in, T* out, int N, int C, int KW, hipStream_t st);
hipError_t launch_add_vec(const float* a, const float* b, float* out, int n, hipStream_t st);

// probs_next_speaker_aggregate on a probs tensor [frames][256] -> out [frames][2]
hipError_t launch_aggregate(const float* probs, int64_t frames, int nb, int from_bin, int to_bin, float* out,
                            hipStream_t st);
// VapGPT.vad post-processing: (p >= cutoff) -> fill silences <= max_fill -> omit spikes <= max_omit
hipError_t launch_vad_post(const float* vad_probs, int B, int Tn, float cutoff, int max_fill, int max_omit, float* out,
                           hipStream_t st);

// bf16 perf mode: fused conv0 -> CN0 -> ReLU -> conv1 -> CN1 -> ReLU (k_conv01.hip).
// c0w: [256][32] bf16 split-bf16 conv0 operand; c0stat: centred Gram statistics (112 floats).
hipError_t launch_conv01(const float* wav, int S, int64_t N, int L0, int L1, const bf16* c0w, const float* c0stat,
                         const float* beta0, const bf16* W1, const bf16* W1s, const float* b1, const float* g1,
                         const float* be1, bf16* out, int64_t out_seq_stride, hipStream_t st, int r0 = 0, int r1 = -1,
                         int grid_cap = 0);
// W [N][K] bf16 -> k-step-major [K/32][N][32] (conv01's W1 stages as contiguous 16 KiB blocks)
hipError_t launch_pack_kstep(const bf16* in, bf16* out, int N, int K, hipStream_t st);
hipError_t read_conv01_stamps(unsigned long long* out);  // diagnostics (VAP_CONV01_STAMPS=1)
hipError_t read_gemm2_stamps(unsigned long long* out);  // diagnostics (VAP_GEMM2_STAMPS=1)
hipError_t read_lstm_stamps(unsigned long long* out);  // diagnostics (VAP_LSTM_STAMPS=1)

// bf16 W [N][K] -> the packed projection layout [N/256][K/32][16][64][8] of the row kernels
// (k_block.hip): one k-step of a 256-wide N tile is 16 KiB contiguous, one wave's 16-row fragment
// 1 KiB in MFMA lane order (k_misc.hip)
hipError_t launch_pack_rowpanel(const bf16* src, bf16* dst, int N, int K, hipStream_t st);

// Fused layer tail (k_block.hip): x' = x + o . Wo^T (skipped when o is null), then
// x = x' + W2 . GELU(W1 . LayerNorm(x')); weights in the packed row-panel layout.
struct BlockArgs {
  float* x;           // residual rows, fp32, in / out
  const bf16* o;      // attention output rows (bf16) or nullptr
  int M;
  int rows_per_seq;   // 0: rows contiguous (stride 256)
  int64_t x_seq;      // sequence strides (elements) of x / o when rows_per_seq > 0
  int64_t o_seq;
  const void* Wo;
  const void* W1;
  const void* W2;
  const float* gamma;
  const float* beta;
  float eps;
  bf16* xb = nullptr;  // optional bf16 copy of the output rows (same row layout as x)
  // optional: the NEXT layer's LayerNorm'd projections from the same rows (np == 3), as lnproj's
  // no-out-projection form: cp = LN2(x) . Wp[0:np)^T (the Q/K/V rows, np x 256 wide), cr = x . Wp[np:np+nr)^T
  // (the raw-row cross K/V, nr x 256 wide); Wp holds the np + nr packed 256-wide tiles back to back; cp / cr
  // rows sit where x's do with the row and sequence strides scaled by np / nr
  const void* Wp = nullptr;
  bf16* cp = nullptr;
  bf16* cr = nullptr;
  const float* gamma2 = nullptr;
  const float* beta2 = nullptr;
  int np = 0, nr = 0;
};
hipError_t launch_block(const BlockArgs& g, int cus, hipStream_t st);
// combinator + vap_head in one launch (k_block.hip heads_kernel): logits [M][256] fp32 of frames
// m = clip * T + t from the bf16 rows x of sequences 2 clip / 2 clip + 1 (row t at x + s x_seq + t 256);
// Wa / Wb / Wh in the packed row-panel layout
struct HeadsArgs {
  const bf16* x;
  int64_t x_seq;
  int M;  // clips x T
  int T;
  const bf16* Wa;
  const bf16* Wb;
  const bf16* Wh;
  const float* gamma;
  const float* beta;
  const float* hbias;
  float* logits;
  float eps;
  const float* vw;  // va_classifier weight [256] / bias [1] -> vad logits [M][2] (speaker 0 / 1)
  const float* vb;
  float* vad;
  int out_T = 0;   // frames per clip of logits / vad (0: T); a frame range's rows go to clip * out_T + out_f0 + t
  int out_f0 = 0;
  const float* xf = nullptr;  // fp32 rows of the same x (layout of x): the VAD head reads them (the reference's
                              // va_classifier takes fp32 x, model.py:257-259); null: the bf16 panels
};
hipError_t launch_heads(const HeadsArgs& g, hipStream_t st);
hipError_t read_block_stamps(unsigned long long* out);
// LayerNorm'd projections of a layer in one launch (k_block.hip): with o, x' = x + o . Wo^T is stored
// to x and cp = LN(x') . Wp^T; without, cp = LN(x) . Wp^T and (nr > 0) cr = x . Wr^T from the raw
// rows.  np / nr = 256-wide N tiles; packed row-panel weights; bf16 outputs.
struct LnProjArgs {
  float* x;
  const bf16* o;
  int M;
  int rows_per_seq;
  int64_t x_seq, o_seq;
  const void* Wo;
  const void* Wp;
  const void* Wr;
  bf16* cp;
  int64_t ldp, cp_seq;
  bf16* cr;
  int64_t ldr, cr_seq;
  const float* gamma;
  const float* beta;
  float eps;
  int np, nr;
};
hipError_t launch_lnproj(const LnProjArgs& g, hipStream_t st);
hipError_t read_lnproj_stamps(unsigned long long* out);
