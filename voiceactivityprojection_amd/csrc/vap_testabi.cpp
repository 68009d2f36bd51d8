// Kernel-level test ABI: every hot-path kernel callable on its own, so tests/test_gpu_kernels.py
// can check each one against a plain PyTorch fp32 reference of the same op.  Not used by the
// engine itself.  precision: VAP_PRECISION_FP32 (storage float) / VAP_PRECISION_BF16 (storage bf16).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "../../include/vap_hip.h"
#include "vap_common.h"
#include "vap_kernels.h"

namespace {
int rc_of(hipError_t e) { return e == hipSuccess ? VAP_OK : VAP_ERR_HIP; }
}  // namespace

namespace {
// one v_mfma_f32_16x16x4_f32 with lane-provided operands: d[lane][r]
__global__ void probe_mfma_f32(const float* a, const float* b, float* d) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[l], b[l], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}
}  // namespace

extern "C" {

int vap_test_probe_mfma_f32(const float* a, const float* b, float* d, void* stream) {
  hipLaunchKernelGGL(probe_mfma_f32, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, d);
  return rc_of(hipGetLastError());
}

int vap_test_gemm(int precision, const void* A, int64_t lda, int64_t a_seq, const void* W, int K, int N,
                  const float* bias, int m_per_seq, int n_seq, void* C, int64_t ldc, int64_t c_seq, const float* add,
                  int64_t ld_add, int64_t add_seq, const float* gamma, const float* beta, int norm, int act,
                  int out_f32, void* stream) {
  GemmArgs g{};
  g.A = A;
  g.lda = lda;
  g.a_seq_stride = a_seq;
  g.W = W;
  g.K = K;
  g.N = N;
  g.bias = bias;
  g.M_per_seq = m_per_seq;
  g.n_seq = n_seq;
  g.C = C;
  g.ldc = ldc;
  g.c_seq_stride = c_seq;
  g.add = add;
  g.ld_add = ld_add;
  g.add_seq_stride = add_seq;
  g.gamma = gamma;
  g.beta = beta;
  g.eps = 1e-5f;
  g.norm = norm;
  g.act = act;
  hipStream_t st = (hipStream_t)stream;
  if (precision == VAP_PRECISION_BF16)
    return rc_of(out_f32 ? launch_gemm<bf16, float>(g, st) : launch_gemm<bf16, bf16>(g, st));
  if (precision == 2) {  // fp32 operands through the split-bf16 kernel (the parity mode's GEMMs): W split here
    void* ws = nullptr;
    if (hipMalloc(&ws, (size_t)N * K * 2 * sizeof(bf16)) != hipSuccess) return VAP_ERR_HIP;
    hipError_t e = launch_split_bf16((const float*)W, (bf16*)ws, (int64_t)N * K, K, st);
    g.W = ws;
    g.split = 1;
    if (e == hipSuccess) e = launch_gemm<float, float>(g, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(ws);
    return rc_of(e);
  }
  return rc_of(launch_gemm<float, float>(g, st));
}

// CPC conv2..4 kernel (k_conv234.hip): W [256][1024] bf16 in the tap-major packing of the engine
// ([n][tap*256 + ci]); repacked k-step major into a scratch buffer here
static unsigned long long* stamps_out = nullptr;  // host buffer for VAP_CONVK4_DBG=16 (vap_test_convk4_stamps)
int vap_test_convk4_stamps(unsigned long long* host) {
  stamps_out = host;
  return VAP_OK;
}
int vap_test_convk4(const void* in, int64_t in_seq, int in_rows, const void* W, const float* bias, const float* gamma,
                    const float* beta, void* out, int64_t out_seq, int M, int S, void* stream) {
  static const int dbg = getenv("VAP_CONVK4_DBG") ? atoi(getenv("VAP_CONVK4_DBG")) : 0;
  hipStream_t st = (hipStream_t)stream;
  void* wks = nullptr;
  if (hipMalloc(&wks, 256 * 1024 * 2) != hipSuccess) return VAP_ERR_HIP;
  int rc = rc_of(launch_pack_kstep((const bf16*)W, (bf16*)wks, 256, 1024, st));
  static unsigned long long* stamps = nullptr;
  if (dbg & 16 && !stamps && hipMalloc(&stamps, 8 * 14 * 8) != hipSuccess) return VAP_ERR_HIP;
  ConvK4Args a{(const bf16*)in, in_seq, in_rows, (const bf16*)wks, bias, gamma, beta, (bf16*)out, out_seq, M, dbg, stamps};
  if (rc == VAP_OK) rc = rc_of(launch_convk4(a, S, st));
  if (hipStreamSynchronize(st) != hipSuccess) rc = VAP_ERR_HIP;
  (void)hipFree(wks);
  if (dbg & 16 && stamps_out && hipMemcpy(stamps_out, stamps, 8 * 14 * 8, hipMemcpyDeviceToHost) != hipSuccess) rc = VAP_ERR_HIP;
  return rc;
}

int vap_test_attention(int precision, const void* Q, int64_t q_ld, int64_t q_seq, const void* K, int64_t k_ld,
                       int64_t k_seq, const void* V, int64_t v_ld, int64_t v_seq, void* O, int64_t o_ld,
                       int64_t o_seq, const float* slopes, int S, int T, int H, int kv_swap, float scale, void* stream) {
  AttnArgs a{Q, q_ld, q_seq, K, k_ld, k_seq, V, v_ld, v_seq, O, o_ld, o_seq, slopes, S, T, H, kv_swap, scale};
  a.split = precision == 2;  // fp32 operands on split-bf16 products (the parity mode's kernel)
  hipStream_t st = (hipStream_t)stream;
  return rc_of(precision == VAP_PRECISION_BF16 ? launch_attention<bf16>(a, st) : launch_attention<float>(a, st));
}

// gx: [S][T][1024] storage type for bf16 (the engine's resident kernel) / fp32 for fp32;
// variant 1 = the L2-streaming bf16 kernel (fp32 gx), 2 the single-CU resident kernel, 3 the pair split,
// 5 the quad split (bf16), 4 the fp32 quad split on split-bf16 operands.  whh_packed: scratch of
// 1024*256 storage elements; out: [S][T][256] storage type.
int vap_test_lstm(int precision, const void* gx, int S, int T, const float* whh, void* whh_packed, void* out,
                  int variant, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (precision == VAP_PRECISION_BF16 && variant == 2) {  // the engine's pre-scaled resident path
    void* gs = nullptr;
    const int64_t n = (int64_t)S * T * 1024;
    if (hipMalloc(&gs, n * sizeof(bf16)) != hipSuccess) return VAP_ERR_HIP;
    hipError_t e = launch_pack_whh_resident(whh, (bf16*)whh_packed, st, true);
    if (e == hipSuccess) e = launch_scale_gates((const bf16*)gx, (bf16*)gs, n, st);
    if (e == hipSuccess)
      e = launch_lstm_resident((const bf16*)gs, S, T, (const bf16*)whh_packed, (bf16*)out, (int64_t)T * 256, st, nullptr,
                               true);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(gs);
    return rc_of(e);
  }
  if (precision == VAP_PRECISION_BF16 && (variant == 3 || variant == 5)) {  // pair split (lstm_pair_kernel) / quad
                                                                             // split (lstm_quadb_kernel), pre-scaled
    void* gs = nullptr;
    void* xb = nullptr;
    const int64_t n = (int64_t)S * T * 1024;
    const size_t xbytes = lstm_pair_xbuf_bytes(S);
    if (hipMalloc(&gs, n * sizeof(bf16)) != hipSuccess) return VAP_ERR_HIP;
    if (hipMalloc(&xb, xbytes) != hipSuccess) {
      (void)hipFree(gs);
      return VAP_ERR_HIP;
    }
    hipError_t e = hipMemsetAsync(xb, 0, xbytes, st);
    if (e == hipSuccess) e = launch_pack_whh_pair(whh, (bf16*)whh_packed, st);
    if (e == hipSuccess) e = launch_scale_gates((const bf16*)gx, (bf16*)gs, n, st);
    void* gp = nullptr;
    const size_t gpb = gx_pair_elems(S, T) * sizeof(bf16);
    if (e == hipSuccess && hipMalloc(&gp, gpb) != hipSuccess) e = hipErrorOutOfMemory;
    if (e == hipSuccess) e = hipMemsetAsync(gp, 0, gpb, st);
    if (e == hipSuccess) e = launch_pack_gx_pair((const bf16*)gs, (bf16*)gp, S, T, st);  // the engine's layout
    if (e == hipSuccess)
      e = launch_lstm_pair((const bf16*)gp, 0, S, T, (const bf16*)whh_packed, (bf16*)out, (int64_t)T * 256, st, nullptr,
                           xb, 1, 0, variant == 5 ? 1 : 0);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (gp) (void)hipFree(gp);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(gs);
    (void)hipFree(xb);
    return rc_of(e);
  }
  if (precision == VAP_PRECISION_FP32 && variant == 4) {  // the quad split on split-bf16 operands (lstm_quad_kernel)
    void* xb = nullptr;
    const size_t xbytes = lstm_quad_xbuf_bytes(S);
    if (hipMalloc(&xb, xbytes) != hipSuccess) return VAP_ERR_HIP;
    void* wq = nullptr;
    if (hipMalloc(&wq, (size_t)2 * 1024 * 256 * sizeof(bf16)) != hipSuccess) {
      (void)hipFree(xb);
      return VAP_ERR_HIP;
    }
    hipError_t e = hipMemsetAsync(xb, 0, xbytes, st);
    if (e == hipSuccess) e = launch_pack_whh_quad(whh, (bf16*)wq, st);
    if (e == hipSuccess)
      e = launch_lstm_quad((const float*)gx, S, T, (const bf16*)wq, (float*)out, (int64_t)T * 256, st, xb, 1, nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(wq);
    (void)hipFree(xb);
    return rc_of(e);
  }
  if (precision == VAP_PRECISION_BF16 && variant == 0) {
    hipError_t e = launch_pack_whh_resident(whh, (bf16*)whh_packed, st);
    if (e != hipSuccess) return VAP_ERR_HIP;
    return rc_of(launch_lstm_resident((const bf16*)gx, S, T, (const bf16*)whh_packed, (bf16*)out, (int64_t)T * 256, st, nullptr));
  }
  if (precision == VAP_PRECISION_BF16) {
    hipError_t e = launch_pack_whh<bf16>(whh, (bf16*)whh_packed, st);
    if (e != hipSuccess) return VAP_ERR_HIP;
    return rc_of(launch_lstm<bf16>((const float*)gx, S, T, (const bf16*)whh_packed, (bf16*)out, (int64_t)T * 256, st));
  }
  hipError_t e = launch_pack_whh<float>(whh, (float*)whh_packed, st);
  if (e != hipSuccess) return VAP_ERR_HIP;
  return rc_of(launch_lstm<float>((const float*)gx, S, T, (const float*)whh_packed, (float*)out, (int64_t)T * 256, st));
}

// out: [2B][L0 + 4][256] storage type (pad rows untouched)
int vap_test_conv0(int precision, const float* wav, int B, int64_t N, int L0, const float* w0, const float* b0,
                   const float* gamma, const float* beta, void* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int64_t seq = (int64_t)(L0 + 4) * 256;
  if (precision == VAP_PRECISION_BF16)
    return rc_of(launch_conv0<bf16>(wav, B, N, L0, w0, b0, gamma, beta, (bf16*)out, seq, st));
  return rc_of(launch_conv0<float>(wav, B, N, L0, w0, b0, gamma, beta, (float*)out, seq, st));
}

int vap_test_layernorm(int precision, const float* x, int64_t rows, const float* gamma, const float* beta, void* out,
                       void* raw, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (precision == VAP_PRECISION_BF16)
    return rc_of(launch_layernorm<bf16>(x, rows, gamma, beta, 1e-5f, (bf16*)out, (bf16*)raw, st));
  return rc_of(launch_layernorm<float>(x, rows, gamma, beta, 1e-5f, (float*)out, (float*)raw, st));
}

int vap_test_pack_weight(const void* W, void* out, int N, int K, void* stream) {
  return rc_of(launch_pack_rowpanel((const bf16*)W, (bf16*)out, N, K, (hipStream_t)stream));
}
int vap_test_read_stamps(unsigned long long* out) { return rc_of(read_conv01_stamps(out)); }
// fused layer tail: x = x' + FFN(LN(x')), x' = x + o . Wo^T (o may be null); plain [N][K] weights
int vap_test_block(float* x, const void* o, int M, const void* Wo, const void* W1, const void* W2, const float* gamma,
                   const float* beta, int cus, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  void* p = nullptr;
  const size_t n1 = 768 * 256, n0 = 256 * 256;
  if (hipMalloc(&p, (2 * n1 + n0) * sizeof(bf16)) != hipSuccess) return VAP_ERR_HIP;
  bf16 *p1 = (bf16*)p, *p2 = p1 + n1, *p0 = p2 + n1;
  hipError_t e = launch_pack_rowpanel((const bf16*)W1, p1, 768, 256, st);
  if (e == hipSuccess) e = launch_pack_rowpanel((const bf16*)W2, p2, 256, 768, st);
  if (e == hipSuccess && Wo) e = launch_pack_rowpanel((const bf16*)Wo, p0, 256, 256, st);
  BlockArgs g{x, (const bf16*)o, M, 0, 0, 0, Wo ? p0 : nullptr, p1, p2, gamma, beta, 1e-5f};
  if (e == hipSuccess) e = launch_block(g, cus, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(p);
  return rc_of(e);
}
// fused combinator + vap_head (k_block.hip heads_kernel): x bf16 [2 B][T][256] (sequence 2b / 2b + 1 =
// speaker 0 / 1 of clip b), plain [256][256] bf16 Wa / Wb / Wh -> logits [B][T][256] fp32
int vap_test_heads(const void* x, int B, int T, const void* Wa, const void* Wb, const void* Wh, const float* gamma,
                   const float* beta, const float* hbias, const float* vw, const float* vb, float* logits, float* vad,
                   void* stream) {
  hipStream_t st = (hipStream_t)stream;
  void* p = nullptr;
  const size_t n0 = 256 * 256;
  if (hipMalloc(&p, 3 * n0 * sizeof(bf16)) != hipSuccess) return VAP_ERR_HIP;
  bf16 *pa = (bf16*)p, *pb = pa + n0, *ph = pb + n0;
  hipError_t e = launch_pack_rowpanel((const bf16*)Wa, pa, 256, 256, st);
  if (e == hipSuccess) e = launch_pack_rowpanel((const bf16*)Wb, pb, 256, 256, st);
  if (e == hipSuccess) e = launch_pack_rowpanel((const bf16*)Wh, ph, 256, 256, st);
  HeadsArgs g{(const bf16*)x, (int64_t)T * 256, B * T, T, pa, pb, ph, gamma, beta, hbias, logits, 1e-5f, vw, vb, vad};
  if (e == hipSuccess) e = launch_heads(g, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(p);
  return rc_of(e);
}
int vap_test_block_packed(float* x, const void* o, int M, const void* Wop, const void* W1p, const void* W2p,
                          const float* gamma, const float* beta, int cus, void* stream) {
  BlockArgs g{x, (const bf16*)o, M, 0, 0, 0, Wop, W1p, W2p, gamma, beta, 1e-5f};
  return rc_of(launch_block(g, cus, (hipStream_t)stream));
}
// fused LN projections (k_block.hip lnproj): plain [N][256] bf16 weights; o != NULL: x' = x + o . Wo^T
// stored to x, cp = LN(x') . Wp^T (np = 1); o == NULL: cp = LN(x) . Wp^T (np = 3), cr = x . Wr^T (nr = 0 / 2)
int vap_test_lnproj(float* x, const void* o, int M, const void* Wo, const void* Wp, int np, const void* Wr, int nr,
                    void* cp, void* cr, const float* gamma, const float* beta, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  void* p = nullptr;
  const size_t n0 = 256 * 256, n1 = (size_t)np * 256 * 256, n2 = (size_t)nr * 256 * 256;
  if (hipMalloc(&p, (n0 + n1 + n2 + 8) * sizeof(bf16)) != hipSuccess) return VAP_ERR_HIP;
  bf16 *p0 = (bf16*)p, *p1 = p0 + n0, *p2 = p1 + n1;
  hipError_t e = hipSuccess;
  if (Wo) e = launch_pack_rowpanel((const bf16*)Wo, p0, 256, 256, st);
  if (e == hipSuccess) e = launch_pack_rowpanel((const bf16*)Wp, p1, np * 256, 256, st);
  if (e == hipSuccess && nr) e = launch_pack_rowpanel((const bf16*)Wr, p2, nr * 256, 256, st);
  LnProjArgs g{};
  g.x = x; g.o = (const bf16*)o; g.M = M; g.Wo = Wo ? p0 : nullptr; g.Wp = p1; g.Wr = nr ? p2 : nullptr;
  g.cp = (bf16*)cp; g.ldp = np * 256; g.cr = (bf16*)cr; g.ldr = nr * 256;
  g.gamma = gamma; g.beta = beta; g.eps = 1e-5f; g.np = np; g.nr = nr;
  if (e == hipSuccess) e = launch_lnproj(g, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(p);
  return rc_of(e);
}
// the same on weights already in the packed layout (vap_test_pack_weight); no allocation, no sync
int vap_test_lnproj_packed(float* x, const void* o, int M, const void* Wop, const void* Wpp, int np, const void* Wrp,
                           int nr, void* cp, void* cr, const float* gamma, const float* beta, void* stream) {
  LnProjArgs g{};
  g.x = x; g.o = (const bf16*)o; g.M = M; g.Wo = o ? Wop : nullptr; g.Wp = Wpp; g.Wr = nr ? Wrp : nullptr;
  g.cp = (bf16*)cp; g.ldp = np * 256; g.cr = (bf16*)cr; g.ldr = nr * 256;
  g.gamma = gamma; g.beta = beta; g.eps = 1e-5f; g.np = np; g.nr = nr;
  return rc_of(launch_lnproj(g, (hipStream_t)stream));
}
int vap_test_read_lnproj_stamps(unsigned long long* out) { return rc_of(read_lnproj_stamps(out)); }
int vap_test_read_block_stamps(unsigned long long* out) { return rc_of(read_block_stamps(out)); }
int vap_test_read_gemm_stamps(unsigned long long* out) { return rc_of(read_gemm2_stamps(out)); }
int vap_test_read_lstm_stamps(unsigned long long* out) { return rc_of(read_lstm_stamps(out)); }
int vap_test_read_lstm_handoff(unsigned long long* out) { return rc_of(read_lstm_handoff(out)); }
int vap_test_read_lstm_xcc(unsigned* out) { return rc_of(read_lstm_xcc(out)); }

}  // extern "C"
