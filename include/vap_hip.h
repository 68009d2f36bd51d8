/* vap_hip.h -- C ABI of the MI355X-native VAP inference engine (libvap_hip.so).
 *
 * The reference (ErikEkstedt/VoiceActivityProjection) has no FFI: its boundary is the Python
 * nn.Module API of vap/model.py.  These entry points are what that API binds to underneath
 * (see INTEGRATION.md for the ctypes binding in voiceactivityprojection_amd/_native.py):
 *
 *   vap_create / vap_set_param / vap_finalize   <- VapGPT(conf) + load_state_dict(sd, strict=True)
 *                                                  (vap/model.py:125-163, run.py:199-201)
 *   vap_forward                                 <- VapGPT.forward(waveform)   (vap/model.py:249-268)
 *   vap_forward_attention                       <- VapGPT.forward(waveform, attention=True)
 *   vap_forward_mono                            <- VapGPTMono.forward(waveform, va, va_history)  (vap/model.py:271-393)
 *   vap_probs + vap_labels_loss                 <- VapGPT.probs(waveform)     (vap/model.py:180-225)
 *   vap_labels_loss                             <- ObjectiveVAP.get_labels + loss_vap (vap/objective.py:209-243)
 *   vap_frame_lengths                           <- the conv length chain (vap/encoder_components.py:83-92,454-460)
 *
 * Conventions: plain pointers and sizes only.  Every tensor argument is a caller-allocated DEVICE
 * buffer (float32 unless stated, C-contiguous).  `stream` is a hipStream_t passed as void*.
 * All calls are asynchronous on `stream` except vap_timing_read.  Return value: VAP_OK or an
 * error code; vap_last_error() gives a message (thread-local).  One handle per model, reentrant
 * across handles.  The forward schedule is fixed at vap_create: the handle reads its developer
 * overrides (VAP_TC_FE / VAP_TC_BE / VAP_BE_SPLIT / VAP_FE_STREAMS / ...) from the
 * environment once, there; the defaults are the product.  Diagnostics builds aside (in-kernel
 * stamps, read once per process), no launch depends on process state after that.
 */
#ifndef VAP_HIP_H
#define VAP_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VAP_OK 0
#define VAP_ERR_INVALID 1     /* bad shape / argument (Python: AssertionError / ValueError) */
#define VAP_ERR_TOO_SHORT 2   /* fewer than horizon+1 frames (Python: RuntimeError, quirk Q2) */
#define VAP_ERR_HIP 3         /* HIP runtime failure */
#define VAP_ERR_WEIGHTS 4     /* unknown key / wrong size / forward before finalize */
#define VAP_ERR_UNSUPPORTED 5 /* configuration outside the kernels' specialisation */

#define VAP_PRECISION_FP32 0  /* parity mode: fp32 storage, v_mfma_f32_16x16x4_f32 */
#define VAP_PRECISION_BF16 1  /* perf mode: bf16 storage, v_mfma_f32_16x16x32_bf16, fp32 accumulate */

/* kernel classes for vap_timing (HIP-event timing of one class inside the timed region) */
#define VAP_K_CONV0 1
#define VAP_K_CONV1 2
#define VAP_K_CONV234 3
#define VAP_K_LSTM_PROJ 4
#define VAP_K_LSTM_REC 5
#define VAP_K_DOWNSAMPLE 6
#define VAP_K_TR_GEMM 7
#define VAP_K_ATTN 8
#define VAP_K_NORM 9
#define VAP_K_HEADS 10
#define VAP_K_PROBS 11

typedef struct vap_dims {
  int dim;            /* VapConfig.dim (must be 256: the CPC encoder width) */
  int num_heads;      /* VapConfig.num_heads (head_dim must be 64) */
  int channel_layers; /* VapConfig.channel_layers */
  int cross_layers;   /* VapConfig.cross_layers */
  int lstm_layers;    /* CPCAR nLevelsGRU (from the state dict) */
  int n_bins;         /* len(VapConfig.bin_times) (must be 4: 256 classes) */
  int precision;      /* VAP_PRECISION_* */
  int mono;           /* 1: VapGPTMono (vap/model.py:271-393): one speaker + VA conditioning, plain GPT stack */
  int va_history_bins;/* VapMonoConfig.va_history_bins when va_history (mono only), else 0 */
} vap_dims;

typedef struct vap_handle vap_handle;

int vap_create(const vap_dims* dims, vap_handle** out);
void vap_destroy(vap_handle* h);

/* State-dict schema: parameter i has reference key `key` and `numel` float32 elements. */
int vap_num_params(const vap_handle* h, int* n);
int vap_param_info(const vap_handle* h, int i, const char** key, int64_t* numel);
/* Copy one parameter (device fp32, reference layout) into the handle. */
int vap_set_param(vap_handle* h, const char* key, const float* src, int64_t numel, void* stream);
/* Repack every parameter into kernel layouts; required after the last vap_set_param. */
int vap_finalize(vap_handle* h, void* stream);

/* lens[0..5] = conv0..conv4 output lengths and the 50 Hz frame count T. */
int vap_frame_lengths(int64_t n_samples, int64_t* lens);
int vap_workspace_size(const vap_handle* h, int batch, int64_t n_samples, size_t* bytes);

/* waveform [B][2][N] -> logits [B][T][256], vad_logits [B][T][2]. */
int vap_forward(vap_handle* h, const float* waveform, int batch, int64_t n_samples, float* logits,
                float* vad_logits, void* workspace, size_t workspace_bytes, void* stream);

/* VapGPT.forward(waveform, attention=True) (vap/model.py:249-268; GPT / GPTStereo attention outputs,
 * vap/modules.py:349-356, 400-407): logits / vad_logits as vap_forward plus the softmax attention
 * weights of every layer, fp32, zeros above the diagonal (causal):
 *   self_attn       [B][2][channel_layers][H][T][T]  ar_channel self attention, speaker 0 / 1
 *   cross_attn      [B][2][cross_layers][H][T][T]    ar cross attention (x1 <- x2, x2 <- x1)
 *   cross_self_attn [B][2][cross_layers][H][T][T]    ar self attention
 * Any of the three may be NULL.  Runs the layer-by-layer schedule (no time chunks). */
int vap_forward_attention(vap_handle* h, const float* waveform, int batch, int64_t n_samples, float* logits,
                          float* vad_logits, float* self_attn, float* cross_attn, float* cross_self_attn,
                          void* workspace, size_t workspace_bytes, void* stream);

/* VapGPTMono.forward(waveform, va, va_history) (vap/model.py:360-393) on a dims.mono handle:
 * waveform [B][1][N], va [B][T][2] (voice activity conditioning), va_history [B][T][bins] or NULL
 * -> logits [B][T][256] (the reference returns `va` itself as "vad").  vap_encode on a mono handle
 * writes [B][T][256]. */
int vap_forward_mono(vap_handle* h, const float* waveform, const float* va, const float* va_history, int batch,
                     int64_t n_samples, float* logits, void* workspace, size_t workspace_bytes, void* stream);
/* VapGPTMono.encode_va (vap/model.py:352-357): out [rows][256] = LN(va_condition(va [rows][2])
 * [+ va_cond_history(va_history [rows][bins])]); va_history may be NULL. */
int vap_encode_va(vap_handle* h, const float* va, const float* va_history, int rows, float* out, void* stream);

/* Rolling-window stream (SURVEY config C5; replaces the reference's per-hop model.probs(x) on a
 * rolled window, sds/run_sds.py:206-241 TurnTakingSDS.add_audio_bytes_to_tensor / run, and the
 * fold loop of run.py:23-131 step_extraction).  The stream owns its window [B][2][window] (zeros
 * at creation) and workspace.  A push rolls `hop` new samples per channel into the window (hop
 * audio [B][2][hop], device) and writes logits [B][T][256] / vad_logits [B][T][2] of the WHOLE
 * window, equal to vap_forward on that window.  In bf16 mode with hop % 160 == 0, the CPC conv rows
 * whose receptive field stays inside the window are carried over from the previous push instead of
 * recomputed (the conv stack is shift-equivariant with stride 160). */
typedef struct vap_stream vap_stream;
int vap_stream_create(vap_handle* h, int batch, int64_t window_samples, int64_t hop_samples, void* stream,
                      vap_stream** out);
int vap_stream_push(vap_stream* s, const float* hop_audio, float* logits, float* vad_logits, void* stream);
/* frames T of a window, window / hop samples, conv4 rows carried over per push, current window (device). */
int vap_stream_info(const vap_stream* s, int* frames, int64_t* window_samples, int64_t* hop_samples,
                    int64_t* reused_rows, const float** window);
/* hipGraph replay of steady-state pushes (bf16 carry-over streams; VAP_STREAM_GRAPH=0 disables): the
 * caller-stream part of a push is captured once per (gate-ring offset, window buffer, output
 * pointers) state and replayed; the recurrence launch stays eager on a side stream.  Reports the
 * graphs captured, the replays so far and the handle's hand-off error word (1 if a flag wait timed
 * out since the last check; synchronous, does not clear it). */
int vap_stream_graphs(vap_stream* s, int* graphs, int64_t* replays, int* handoff_error);
/* Window back to zeros; the next push recomputes every row. */
int vap_stream_reset(vap_stream* s, void* stream);
void vap_stream_destroy(vap_stream* s);

/* EncoderCPC.encode_audio (vap/model.py:169-175): out [2][B][T][256] = (x1, x2). */
int vap_encode(vap_handle* h, const float* waveform, int batch, int64_t n_samples, float* out, void* workspace,
               size_t workspace_bytes, void* stream);

/* ObjectiveVAP.probs_next_speaker_aggregate (vap/objective.py:184-204): probs [B][T][256] -> out [B][T][2]. */
int vap_aggregate(const float* probs, int batch, int frames, int n_bins, int from_bin, int to_bin, float* out,
                  void* stream);

/* VapGPT.vad post-processing (vap/model.py:227-247, vap/utils.py:239-272): binarise
 * sigmoid(vad_logits [B][T][2]) >= cutoff, fill silences of <= max_fill_frames, then omit spikes of
 * <= max_omit_frames -> out (0/1 floats). */
int vap_vad_postprocess(const float* vad_logits, int batch, int frames, float cutoff, int max_fill_frames,
                        int max_omit_frames, float* out, void* stream);

/* probs() epilogue: probs [B][T][256], vad = sigmoid [B][T][2], p_now / p_future [B][T][2], H [B][T]. */
int vap_probs(const float* logits, const float* vad_logits, int batch, int frames, int n_bins, int now0, int now1,
              int fut0, int fut1, float* probs, float* vad, float* p_now, float* p_future, float* H, void* stream);

/* labels [B][T - horizon] (int64) from voice activity va [B][T][2], and the per-frame VAP cross
 * entropy loss [B][T - horizon] of logits [B][T][256] against them (logits and loss may both be
 * NULL: labels only).  bin_frames is a HOST array of n_bins frame counts (bin_times_to_frames,
 * vap/objective.py:10-11). */
/* VapGPT.probs epilogue in one call (vap/model.py:180-225): vap_probs' outputs plus labels [B][T-h] and
 * loss [B][T-h] of vap_labels_loss, with the labels taken from sigmoid(vad_logits) (quirk Q1); h = the
 * sum of bin_frames (at most 128).  Same values as vap_probs followed by vap_labels_loss on its vad. */
int vap_probs_loss(const float* logits, const float* vad_logits, int batch, int frames, int n_bins, int now0, int now1,
                   int fut0, int fut1, const int* bin_frames, float threshold, float* probs, float* vad, float* p_now,
                   float* p_future, float* H, int64_t* labels, float* loss, void* stream);
int vap_labels_loss(const float* logits, const float* va, int batch, int frames, const int* bin_frames, int n_bins,
                    float threshold, int64_t* labels, float* loss, void* stream);

/* Wait for `stream` (the caller's stream of the last call on h) and report a hand-off failure of
 * the calls since the last check: VAP_ERR_HIP when a bounded flag wait of the persistent LSTM
 * recurrence or of a captured stream push timed out (~2 s; their outputs are then invalid).
 * Without it such a failure is reported by the next vap_forward / vap_forward_mono / vap_encode /
 * vap_stream_push on the handle (a host read of a mapped word, no device sync). */
int vap_synchronize(vap_handle* h, void* stream);

/* Timing hook: record HIP events around every launch of kernel class `cls` (0 = off); -cls times
 * the class with the time-pipelined front end on the caller stream only (no second stream). */
int vap_timing(vap_handle* h, int cls);
/* Synchronises the recorded events; total device milliseconds and launch count since last read. */
int vap_timing_read(vap_handle* h, double* total_ms, int* launches);

const char* vap_last_error(void);
const char* vap_build_info(void);

/* ---- kernel-level test ABI (tests/test_gpu_kernels.py): each hot-path kernel on its own. ----
 * Storage-type buffers are float (VAP_PRECISION_FP32) or bf16 (VAP_PRECISION_BF16). */
int vap_test_gemm(int precision, const void* A, int64_t lda, int64_t a_seq, const void* W, int K, int N,
                  const float* bias, int m_per_seq, int n_seq, void* C, int64_t ldc, int64_t c_seq, const float* add,
                  int64_t ld_add, int64_t add_seq, const float* gamma, const float* beta, int norm, int act,
                  int out_f32, void* stream);
int vap_test_attention(int precision, const void* Q, int64_t q_ld, int64_t q_seq, const void* K, int64_t k_ld,
                       int64_t k_seq, const void* V, int64_t v_ld, int64_t v_seq, void* O, int64_t o_ld,
                       int64_t o_seq, const float* slopes, int S, int T, int H, int kv_swap, float scale, void* stream);
int vap_test_lstm(int precision, const void* gx, int S, int T, const float* whh, void* whh_packed, void* out,
                  int variant, void* stream);
int vap_test_conv0(int precision, const float* wav, int B, int64_t N, int L0, const float* w0, const float* b0,
                   const float* gamma, const float* beta, void* out, void* stream);
/* one v_mfma_f32_16x16x4_f32 with lane-provided operands a[64], b[64] -> d[64][4] (layout probe) */
int vap_test_probe_mfma_f32(const float* a, const float* b, float* d, void* stream);
int vap_test_layernorm(int precision, const float* x, int64_t rows, const float* gamma, const float* beta, void* out,
                       void* raw, void* stream);
/* weight packing into the projection layout [N/256][K/32][16][64][8] (N % 256 == 0, K % 32 == 0) */
int vap_test_pack_weight(const void* W, void* out, int N, int K, void* stream);
/* fused layer tail (bf16 path): x' = x + o . Wo^T (o [M][256] bf16, skipped when o is NULL), then
 * x = x' + W2 . GELU(W1 . LayerNorm(x')); plain [N][K] bf16 weights; cus picks the rows per workgroup */
int vap_test_block(float* x, const void* o, int M, const void* Wo, const void* W1, const void* W2, const float* gamma,
                   const float* beta, int cus, void* stream);
/* fused LayerNorm'd projections (bf16 path), plain [N][256] bf16 weights: with o (np = 1):
 * x' = x + o . Wo^T is stored to x and cp [M][256] = LN(x') . Wp^T; without o (np = 3):
 * cp [M][768] = LN(x) . Wp^T and, nr = 2, cr [M][512] = x . Wr^T from the raw rows */
int vap_test_lnproj(float* x, const void* o, int M, const void* Wo, const void* Wp, int np, const void* Wr, int nr,
                    void* cp, void* cr, const float* gamma, const float* beta, void* stream);
/* the same with weights already packed (vap_test_pack_weight): no allocation, no synchronisation */
int vap_test_lnproj_packed(float* x, const void* o, int M, const void* Wop, const void* Wpp, int np, const void* Wrp,
                           int nr, void* cp, void* cr, const float* gamma, const float* beta, void* stream);
/* fused combinator + vap_head (bf16 path, k_block.hip heads_kernel): x bf16 [2B][T][256] (sequences 2b / 2b+1 =
 * the two speakers of clip b), plain [256][256] bf16 Wa / Wb / Wh -> logits [B][T][256] fp32 =
 * (GELU(LN(x1 Wa^T)) + GELU(LN(x2 Wb^T))) Wh^T + hbias, vad [B][T][2] = x1 / x2 . vw + vb */
int vap_test_heads(const void* x, int B, int T, const void* Wa, const void* Wb, const void* Wh, const float* gamma,
                   const float* beta, const float* hbias, const float* vw, const float* vb, float* logits, float* vad,
                   void* stream);
/* the same with weights already packed (vap_test_pack_weight) */
int vap_test_block_packed(float* x, const void* o, int M, const void* Wop, const void* W1p, const void* W2p,
                          const float* gamma, const float* beta, int cus, void* stream);
/* workspace plan of a forward (diagnostics): byte offsets of X1..X4 (conv1..4 rows), GX (gate rows),
 * H0 (LSTM h), X (residual stream), the total, then the per-sequence strides s1..s4, sh (elements) */
int vap_test_plan(const vap_handle* h, int batch, int64_t n_samples, int64_t* out);
/* pair-recurrence exchange tag counter of a handle (tests): *get = the last tag issued; set >= 0 moves it (e.g.
 * next to the 32-bit wrap, which the next launch handles by clearing the exchange slots) */
int vap_test_xtag(vap_handle* h, int64_t set, int64_t* get);
/* robustness tests: from now on the handle never publishes the recurrence's ready flag of time chunk `chunk`
 * (-1: publish all again), so the bounded wait times out and the hand-off error surfaces */
int vap_test_drop_ready(vap_handle* h, int chunk);
/* pair-recurrence exchange store policy of a handle (VAP_LSTM_XPLAIN at vap_create): 0 by XCD handshake,
 * 1 plain (L2) stores always, -1 write-through always */
int vap_test_lstm_xplain(vap_handle* h, int policy);
/* timing diagnostics: 8 x 24 s_memtime stamps of sampled conv01 workgroups (VAP_CONV01_STAMPS=1) */
int vap_test_read_stamps(unsigned long long* out);
/* timing diagnostics: 8 x 24 s_memtime stamps of sampled fused-block workgroups (VAP_BLOCK_STAMPS=1) */
int vap_test_read_block_stamps(unsigned long long* out);
/* timing diagnostics: 8 x 24 s_memtime stamps of sampled LN-projection workgroups (VAP_LNPROJ_STAMPS=1) */
int vap_test_read_lnproj_stamps(unsigned long long* out);
/* timing diagnostics: 8 x 2 x 4 x 6 s_memtime stamps of sampled bf16 GEMM k-steps (VAP_GEMM2_STAMPS=1) */
int vap_test_read_gemm_stamps(unsigned long long* out);  /* + 8 x 6 tile-phase stamps after the 8 x 2 x 4 x 6 */
/* CPC conv2..4 slab kernel (k_conv234.hip) on its own: conv k4 s2 256->256 + bias + ChannelNorm + ReLU.
 * in: bf16 rows [S][in_seq] with one zero pad row in front (output t reads buffer rows 2t .. 2t+3), in_rows
 * readable; W [256][1024] bf16 in the engine's tap-major packing ([n][tap*256 + ci]); out rows [S][out_seq], M per sequence */
int vap_test_convk4(const void* in, int64_t in_seq, int in_rows, const void* W, const float* bias, const float* gamma,
                    const float* beta, void* out, int64_t out_seq, int M, int S, void* stream);
/* timing diagnostics: host buffer that receives 8 x 12 phase stamps of the next vap_test_convk4 (VAP_CONVK4_DBG=16) */
int vap_test_convk4_stamps(unsigned long long* host);
/* timing diagnostics: 8 x 4 x 5 s_memtime stamps of bf16 LSTM steps 100..103 (VAP_LSTM_STAMPS=1) */
int vap_test_read_lstm_stamps(unsigned long long* out);
/* timing diagnostics (VAP_LSTM_HANDOFF=1): s_memrealtime (100 MHz) of the last pair recurrence's workgroup 0:
 * out[0] launch start, then per time chunk c: out[1+3c] ready wait begins, out[2+3c] ready seen,
 * out[3+3c] done published (49 values) */
int vap_test_read_lstm_handoff(unsigned long long* out);
/* XCD handshake of the last pair-LSTM launch, blocks 0..63: own XCC id | partner's << 8 | exchange
   kept in L2 << 16 | 1 << 24 (written) */
int vap_test_read_lstm_xcc(unsigned* out);

#ifdef __cplusplus
}
#endif
#endif
