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
#include <cstdlib>
#include <type_traits>

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

VAP_DEV float cell_sig(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
VAP_DEV float cell_tanh(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x)); }

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

  const float* gxs = gx + (int64_t)(valid ? seq : 0) * Tn * G4 + 64 * w + (lane >> 4) * 4;
  // this wave's packed W_hh fragments through a buffer resource: one lane offset, scalar fragment
  // offsets (a pointer per fragment would hold 2 VGPRs for each of the 16 KG fragments)
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(whh + (int64_t)w * 16 * Gm::KG * 64, 16u * Gm::KG * 64u * 16u);
  const uint32_t wlo = (uint32_t)lane * 16u;
  // W_hh does not change between steps, so its fragments stream through a register ring of PD
  // k-groups that runs on across the step boundary (the fragments of k-group kg are re-issued as
  // soon as k-group kg is consumed, for the next step), and the gate rows gx of step t+1 load
  // while step t computes: no L2 / HBM round trip is exposed per k-group or per step (the
  // load-then-use form ran ~47 us per step at 2 workgroups per launch).
  constexpr int KG = Gm::KG, PD = sizeof(T) == 4 ? 4 : 2;  // fp32: 465 registers, no spills
  static_assert(KG % PD == 0, "the ring slot of a k-group must repeat across steps");
  chunk16 wr[PD][16];
  auto wload = [&](int kg, chunk16(&r)[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = buf_load16(rw, wlo, (uint32_t)((i * KG + kg) * 64 * 16));
  };
#pragma unroll
  for (int p = 0; p < PD; ++p) wload(p, wr[p]);
  f32x4 gxn[4][4];
  auto gxload = [&](int t) {
    const float* gxt = gxs + (int64_t)t * G4;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int ut = 0; ut < 4; ++ut)
        gxn[g][ut] = valid ? *(const f32x4*)(gxt + g * HD + ut * 16) : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  gxload(0);
  for (int t = 0; t < Tn; ++t) {
    const unsigned char* hcur = hbuf[t & 1];
    unsigned char* hnext = hbuf[(t + 1) & 1];
    f32x4 acc[4][4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int ut = 0; ut < 4; ++ut) acc[g][ut] = gxn[g][ut];
    gxload(t + 1 < Tn ? t + 1 : t);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
      const chunk16 hb = *(const chunk16*)(hcur + (lane & 15) * Gm::HROW + (kg * 4 + (lane >> 4)) * 16);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int ut = 0; ut < 4; ++ut) acc[g][ut] = mfma_chunk<T>(wr[kg % PD][g * 4 + ut], hb, acc[g][ut]);
      wload((kg + PD) % KG, wr[kg % PD]);
      __builtin_amdgcn_sched_barrier(0);  // keep the ring: no load hoisted past its k-group
    }
    // cell update: unit u = 64w + 16ut + (lane>>4)*4 + r, sequence lane&15
#pragma unroll
    for (int ut = 0; ut < 4; ++ut) {
      float h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // v_exp / v_rcp forms (abs. error ~2e-7; libm expf / tanhf cost ~4 us a step)
        const float ig = cell_sig(acc[0][ut][r]);
        const float fg = cell_sig(acc[1][ut][r]);
        const float gg = cell_tanh(acc[2][ut][r]);
        const float og = cell_sig(acc[3][ut][r]);
        c[ut][r] = fg * c[ut][r] + ig * gg;
        h[r] = og * cell_tanh(c[ut][r]);
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

// ------------------------------------------------------------------------------------------
// bf16 perf mode: W_hh RESIDENT on the CU.  512 KiB bf16 = 4 waves (one per SIMD, 512-register
// budget each) x 128 fragments of 1 KiB: 90 per wave in registers, 38 per wave in LDS (152 KiB),
// so a step reads no weights from L2/HBM.  Wave w owns units [64w, 64w+64): row tiles
// rt = g*4 + ut (rows g*256 + 64w + 16ut + lane&15), k-groups kg (k = 32kg + 8(lane>>4) + e),
// fragment f = rt*8 + kg.  h_{t-1} lives in an 8 KiB LDS image [seq][256] with chunk ^= seq
// (conflict-free b128 reads).  gx (bf16) of step t+1 is prefetched while step t computes.
// ------------------------------------------------------------------------------------------
constexpr int R_NW = 4, R_NF = 128, R_NAGPR = 64, R_NVGPR = 26, R_NREG = R_NAGPR + R_NVGPR, R_NLDS = R_NF - R_NREG;

VAP_DEV float fsig(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
VAP_DEV float ftanh(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x)); }

// MFMA with the A operand in AGPRs / VGPRs, issued as inline asm so the compiler keeps the
// weight fragments resident in the accumulator file instead of spilling/copying them per use.
// hipcc pads no hazards inside asm: LEAD adds the VALU-write -> MFMA-srcC wait (s_nop 1); TAIL
// adds the MFMA-D -> VALU-read wait (16 states) after the last MFMA of a block.
// The waits live INSIDE the MFMA's asm string: a separate "s_nop" statement has no operands, so
// the compiler may legally schedule the VALU consumer of the MFMA output ahead of it (observed:
// stale accumulators on some lanes).
#define VAP_MFMA_ASM(LEAD, TAIL, ACON)                                                              \
  do {                                                                                             \
    if constexpr (LEAD && TAIL)                                                                    \
      asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\ts_nop 15"                 \
                   : "+v"(c) : ACON(a), "v"(b));                                                    \
    else if constexpr (LEAD)                                                                       \
      asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : ACON(a), "v"(b)); \
    else if constexpr (TAIL)                                                                       \
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\ts_nop 15" : "+v"(c) : ACON(a), "v"(b)); \
    else                                                                                           \
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : ACON(a), "v"(b));         \
  } while (0)

template <int LEAD, int TAIL>
VAP_DEV void mfma_a(f32x4& c, const chunk16& a, const chunk16& b) {
  VAP_MFMA_ASM(LEAD, TAIL, "a");
}
template <int LEAD, int TAIL>
VAP_DEV void mfma_v(f32x4& c, const chunk16& a, const chunk16& b) {
  VAP_MFMA_ASM(LEAD, TAIL, "v");
}

// One cell of the LSTM update for register r of a finished unit tile.
// PRE: the gate pre-activations arrive pre-scaled (W_ih, W_hh, biases packed with -log2e on the i / f
// / o rows and 2 log2e on the g rows), and c is kept as 2 log2e c, so every activation is
// exp2 + add + rcp with no argument scaling: 10 VALU + 10 transcendentals per cell instead of 15 + 10.
constexpr float KC = 2.8853900817779268f;  // 2 log2(e)
template <bool PRE>
VAP_DEV void lstm_cell(const f32x4 (&acc)[4], int r, float& c, float& h) {
  if constexpr (PRE) {
    auto sg = [](float x) { return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x)); };  // sigmoid(-x ln2)
    const float ig = sg(acc[0][r]), fg = sg(acc[1][r]), og = sg(acc[3][r]);
    const float gk = __builtin_fmaf(-2.0f * KC, sg(acc[2][r]), KC);  // 2 log2e tanh(g), acc = 2 log2e g
    c = fg * c + ig * gk;                                               // 2 log2e c
    h = og * __builtin_fmaf(-2.0f, sg(c), 1.0f);                        // tanh(c) = 1 - 2 / (1 + 2^{c'})
  } else {
    const float ig = fsig(acc[0][r]), fg = fsig(acc[1][r]), gg = ftanh(acc[2][r]), og = fsig(acc[3][r]);
    c = fg * c + ig * gg;
    h = og * ftanh(c);
  }
}

// LDS operands of one k-step q = ut*8 + kg: the h fragment and the LDS-resident weight fragments
// (gate 3 always, gate 2 for the last ones).  Gates 0/1 live in AGPRs, gate 2 mostly in VGPRs.
struct KPre {
  chunk16 hf, w2, w3;
};

template <int Q>
VAP_DEV void kload(KPre& p, const chunk16* wl, const unsigned char* hb, int sl, int lane) {
  constexpr int UT = Q >> 3, KG = Q & 7;
  constexpr int F2 = (2 * 4 + UT) * 8 + KG, F3 = (3 * 4 + UT) * 8 + KG;
  p.hf = *(const chunk16*)(hb + sl * 512 + (((KG * 4 + (lane >> 4)) ^ sl) << 4));
  if constexpr (F2 >= R_NREG) p.w2 = wl[(F2 - R_NREG) * 64];
  if constexpr (F3 >= R_NREG) p.w3 = wl[(F3 - R_NREG) * 64];
}

template <int F, int LEAD, int TAIL>
VAP_DEV void mfma_f(f32x4& c, const chunk16 (&wa)[R_NAGPR], const chunk16 (&wv)[R_NVGPR], const chunk16& lds,
                    const chunk16& hf) {
  if constexpr (F < R_NAGPR)
    mfma_a<LEAD, TAIL>(c, wa[F], hf);
  else if constexpr (F < R_NREG)
    mfma_v<LEAD, TAIL>(c, wv[F - R_NAGPR], hf);
  else
    mfma_v<LEAD, TAIL>(c, lds, hf);
}

struct LstmState {
  bf16x4 gn[4][4];  // gx of the next step (prefetched)
  float c[4][4];    // cell state: unit 64w + 16ut + 4(lane>>4) + r, sequence lane&15
  float hv[4][4];   // h_t of this step
  f32x4 acc[4], prev[4];
};

// k-step Q of the step: issue the LDS reads of step Q+1, then the four MFMAs of step Q; the cell
// update of the previous unit tile is interleaved (one register per two k-steps) so the vector
// and matrix pipes of the SIMD overlap.
template <int Q, bool PRE>
VAP_DEV void kstep(LstmState& st, const KPre& cur, KPre& nxt, const bf16* gt, const chunk16 (&wa)[R_NAGPR],
                   const chunk16 (&wv)[R_NVGPR], const chunk16* wl, const unsigned char* hb, int sl, int lane) {
  constexpr int UT = Q >> 3, KG = Q & 7;
  if constexpr (KG == 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      st.acc[g] = f32x4{(float)st.gn[UT][g][0], (float)st.gn[UT][g][1], (float)st.gn[UT][g][2],
                        (float)st.gn[UT][g][3]};
      st.gn[UT][g] = *(const bf16x4*)(gt + g * HD + UT * 16);  // prefetch step t+1
    }
  }
  if constexpr (Q + 1 < 32) kload<Q + 1>(nxt, wl, hb, sl, lane);
  constexpr int LEAD = KG == 0 ? 1 : 0;
  constexpr int TAIL = (UT == 3 && KG == 7) ? 1 : 0;  // only the last tile's results are read right away
  mfma_f<(0 * 4 + UT) * 8 + KG, LEAD, TAIL>(st.acc[0], wa, wv, cur.w2, cur.hf);
  mfma_f<(1 * 4 + UT) * 8 + KG, LEAD, TAIL>(st.acc[1], wa, wv, cur.w2, cur.hf);
  mfma_f<(2 * 4 + UT) * 8 + KG, LEAD, TAIL>(st.acc[2], wa, wv, cur.w2, cur.hf);
  mfma_f<(3 * 4 + UT) * 8 + KG, LEAD, TAIL>(st.acc[3], wa, wv, cur.w3, cur.hf);
  if constexpr (UT > 0) {
    if constexpr (KG == 1)  // consumers of the previous tile stay below this point (no MFMA->VALU hazard)
      asm volatile("" : "+v"(st.prev[0]), "+v"(st.prev[1]), "+v"(st.prev[2]), "+v"(st.prev[3]));
    if constexpr (KG & 1) {
      lstm_cell<PRE>(st.prev, KG >> 1, st.c[UT - 1][KG >> 1], st.hv[UT - 1][KG >> 1]);
      // pin the cell here, between this k-step's MFMAs and the next's (all volatile asm): left
      // alone the compiler sinks every cell update to the h write after the step's MFMAs, so the
      // transcendental work never overlaps the matrix pipe
      asm volatile("" : "+v"(st.c[UT - 1][KG >> 1]), "+v"(st.hv[UT - 1][KG >> 1]));
    }
  }
  if constexpr (KG == 7) {
#pragma unroll
    for (int g = 0; g < 4; ++g) st.prev[g] = st.acc[g];
    if constexpr (UT == 3) {
#pragma unroll
      for (int r = 0; r < 4; ++r) lstm_cell<PRE>(st.prev, r, st.c[3][r], st.hv[3][r]);
    }
  }
}

template <int Q, bool PRE>
VAP_DEV void ksteps(LstmState& st, KPre& cur, KPre& nxt, const bf16* gt, const chunk16 (&wa)[R_NAGPR],
                    const chunk16 (&wv)[R_NVGPR], const chunk16* wl, const unsigned char* hb, int sl, int lane) {
  kstep<Q, PRE>(st, cur, nxt, gt, wa, wv, wl, hb, sl, lane);
  if constexpr (Q + 1 < 32) ksteps<Q + 1, PRE>(st, nxt, cur, gt, wa, wv, wl, hb, sl, lane);
}

// diagnostics (VAP_LSTM_STAMPS=1): wave 0 of workgroups 0..7 records s_memtime at steps 100..103:
// [step start, k-steps + cell done, after barrier 1, h written, after barrier 2]
__device__ unsigned long long g_lstm_stamps[8][4][5];

template <bool ST, bool PRE>
__global__ __launch_bounds__(256, 1) void lstm_resident_kernel(const bf16* __restrict__ gx, int S, int Tn,
                                                              const chunk16* __restrict__ wp, bf16* __restrict__ out,
                                                              int64_t out_seq_stride, LstmSync sync) {
  __shared__ __attribute__((aligned(16))) chunk16 wls[R_NW * R_NLDS * 64];
  __shared__ __attribute__((aligned(16))) unsigned char hb[NS * 512];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int sl = lane & 15;  // sequence within the group (MFMA column)
  const int seq = blockIdx.x * NS + sl;
  const bool valid = seq < S;

  chunk16 wa[R_NAGPR], wv[R_NVGPR];
  const chunk16* wsrc = wp + (int64_t)w * R_NF * 64 + lane;
#pragma unroll
  for (int f = 0; f < R_NAGPR; ++f) wa[f] = wsrc[f * 64];
#pragma unroll
  for (int f = 0; f < R_NVGPR; ++f) wv[f] = wsrc[(R_NAGPR + f) * 64];
  chunk16* wl = wls + w * R_NLDS * 64 + lane;
#pragma unroll
  for (int f = 0; f < R_NLDS; ++f) wl[f * 64] = wsrc[(R_NREG + f) * 64];
  for (int i = tid; i < NS * 512 / 4; i += 256) ((unsigned*)hb)[i] = 0u;
  // ranges covered by this workgroup's sequences (persistent multi-range launch)
  int ra = 0, rb = -1;
  if (sync.ready) {
    if (sync.time_mode) {
      rb = 0;  // time chunks: the first chunk now, the others at their boundaries
    } else {
      const int s_first = blockIdx.x * NS, s_last = min(S, s_first + NS) - 1;
      while (sync.seq_end[ra] <= s_first) ++ra;
      rb = ra;
      while (sync.seq_end[rb] <= s_last) ++rb;
    }
    if (tid == 0) {
      // the producer stream publishes ready[r] after the range's gate projection completed (its
      // kernel boundary wrote the rows back).  Poll RELAXED (L2-served sc1 loads), then ONE
      // agent-scope acquire (invalidates this CU's L1; the vmcnt wait holds the barrier until it has
      // completed).  Never poll with system-scope acquires: each one is a `buffer_inv sc0 sc1`, and
      // ~100 workgroups issuing them back to back corrupted the outputs of the conv / GEMM kernels
      // running beside them (rows of sequence 0 at batch >= 640 x 2.5 s).
      // Bounded: after ~2 s (100 MHz s_memrealtime) give up, flag the error word and run on, so a
      // lost flag can never hang the device (done counters are still published below)
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (int r = ra; r <= rb; ++r)
        while (__hip_atomic_load(sync.ready + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < sync.epoch) {
          __builtin_amdgcn_s_sleep(8);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
            if (sync.error) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
        }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  LstmState st;
#pragma unroll
  for (int ut = 0; ut < 4; ++ut)
#pragma unroll
    for (int r = 0; r < 4; ++r) st.c[ut][r] = 0.f;

  const bf16* gxs = gx + (int64_t)(valid ? seq : 0) * Tn * G4 + 64 * w + (lane >> 4) * 4;
  const int goff = sync.gx_off;
  auto grow = [&](int t) -> int64_t {  // gate row of step t (a ring when gx_off != 0)
    const int r = t + goff;
    return (int64_t)(r >= Tn ? r - Tn : r) * G4;
  };
#pragma unroll
  for (int ut = 0; ut < 4; ++ut)
#pragma unroll
    for (int g = 0; g < 4; ++g) st.gn[ut][g] = *(const bf16x4*)(gxs + grow(0) + g * HD + ut * 16);
  __syncthreads();

  KPre pa, pb;
  int chunk = 0;
  const bool samp = ST && blockIdx.x < 8 && tid == 0;
  auto stamp = [&](int t, int k) {
    if constexpr (ST) {
      const unsigned long long v = __builtin_amdgcn_s_memtime();
      if (samp && t >= 100 && t < 104) g_lstm_stamps[blockIdx.x][t - 100][k] = v;
    }
  };
  for (int t = 0; t < Tn; ++t) {
    const bf16* gt = gxs + grow(t + 1 < Tn ? t + 1 : t);
    stamp(t, 0);
    kload<0>(pa, wl, hb, sl, lane);
    ksteps<0, PRE>(st, pa, pb, gt, wa, wv, wl, hb, sl, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp(t, 1);
    __builtin_amdgcn_s_barrier();  // every wave has consumed h_{t-1} (no vmcnt drain: gx prefetch stays in flight)
    stamp(t, 2);
#pragma unroll
    for (int ut = 0; ut < 4; ++ut) {
      const int u = 64 * w + 16 * ut + (lane >> 4) * 4;
      bf16x4 hv4 = {(bf16)st.hv[ut][0], (bf16)st.hv[ut][1], (bf16)st.hv[ut][2], (bf16)st.hv[ut][3]};
      *(bf16x4*)(hb + sl * 512 + (((u >> 3) ^ sl) << 4) + (u & 7) * 2) = hv4;
      if (valid) *(bf16x4*)(out + (int64_t)seq * out_seq_stride + (int64_t)t * HD + u) = hv4;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stamp(t, 3);
    __builtin_amdgcn_s_barrier();  // h_t visible to every wave
    stamp(t, 4);
    if (sync.time_mode && chunk < sync.nr && t + 1 >= sync.seq_end[chunk]) {
      // end of a time chunk: publish its h rows (every chunk ending here), then wait for the next
      // chunk's gate projection
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int c0 = chunk;
      while (chunk < sync.nr && t + 1 >= sync.seq_end[chunk]) ++chunk;
      if (tid == 0) {
        // release: write this XCD's L2 back (the h rows of every wave, drained above), then the
        // counters (the consumer stream's wait-value and kernels read memory)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int c = c0; c < chunk; ++c)
          __hip_atomic_fetch_add(sync.done + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (chunk < sync.nr) {  // relaxed poll + one agent acquire, as at the start
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          while (__hip_atomic_load(sync.ready + chunk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < sync.epoch) {
            __builtin_amdgcn_s_sleep(8);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
              if (sync.error) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              break;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      if (chunk < sync.nr) {
        __syncthreads();
        // the in-step prefetch of step t+1 may predate the projection: load it again
        const bf16* gn1 = gxs + grow(t + 1);
#pragma unroll
        for (int ut = 0; ut < 4; ++ut)
#pragma unroll
          for (int g = 0; g < 4; ++g) st.gn[ut][g] = *(const bf16x4*)(gn1 + g * HD + ut * 16);
      }
    }
  }
  if (sync.ready && !sync.time_mode) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's h stores are complete
    __syncthreads();
    if (tid == 0) {  // release: the consumer stream's kernels (any XCD) see every h of these ranges
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int r = ra; r <= rb; ++r) __hip_atomic_fetch_add(sync.done + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------------------------------
// W_hh split over a PAIR of workgroups: two CUs per 16 sequences.
//
// The single-CU kernel above is issue-bound on one SIMD: per step each wave issues 128 MFMAs and 16
// cells (10 transcendentals each) per lane with no second wave to hide latency (~3.4 us per step
// beside the other kernels, 2000 dependent steps per 20 s clip: the recurrence is the critical
// chain of the time-pipelined forward).  Here workgroup half p of a pair owns hidden units
// [128p, 128p + 128): 4 gates x 128 units = 512 W_hh rows = 256 KiB bf16, held entirely in registers
// by 8 waves (2 per SIMD, 32 fragments each); wave w owns units 128p + 16w .. +16 (one row tile per
// gate, 32 MFMAs and 4 cells per lane per step).  Each step needs the partner's half of h_{t-1}:
//   * every lane publishes its 4 h values (units 128p + 16w + 4(lane>>4) + r, sequence lane&15) as
//     two 8-byte {2 x bf16, tag} granules in ONE 16-byte write-through (sc1) store into the pair's
//     exchange slot for step parity t&1; tag = (launch epoch, step);
//   * the same lane of the partner polls that 16-byte slot with sc1 loads until both tags match
//     (no separate flag: the data carries its own readiness; a granule is never torn), then writes
//     the 4 values into its LDS image of h;
//   * the poll is issued before this half's own-unit k-steps (half of the MFMAs), so most of the
//     exchange latency overlaps them; one barrier publishes the partner's half, a second the own h_t.
// Two parity slots suffice: a half can write h_t only after reading the partner's h_{t-1}, which the
// partner published only after reading our h_{t-2} (the slot being overwritten).
// Pairs are blocks (b, b+8) of each 16-block group (same XCD under round-robin placement: speed
// only); every spin is bounded (~2 s, then the error word is set and the step runs on).
// ------------------------------------------------------------------------------------------
constexpr int P_NW = 8, P_NF = 32;  // waves per workgroup, W fragments per wave (4 gates x 8 k-steps)
constexpr int P_SLOT = 2 * 2 * 512;  // 16-byte exchange slots per pair: [half][parity][lane of the workgroup]

VAP_DEV u32x4 xload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);  // sc1: L2-coherent, bypasses L1
}

__device__ unsigned long long g_lstm_handoff[1 + 3 * 16];
__device__ unsigned g_lstm_xcc[64];  // block b < 64 of the last launch: own XCC | partner's << 8 | L2 exchange << 16 | 1 << 24

template <bool PRE, bool ST>
__global__ __launch_bounds__(512, 2) void lstm_pair_kernel(const bf16* __restrict__ gx, int seq0, int S, int Tn,
                                                          const chunk16* __restrict__ wp, bf16* __restrict__ out,
                                                          int64_t out_seq_stride, LstmSync sync, u32x4* xbuf) {
  __shared__ __attribute__((aligned(16))) unsigned char hb[NS * 512];  // h_{t-1} [seq][256], chunk ^= seq
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x;
  const int grp = (b >> 4) * 8 + (b & 7), p = (b >> 3) & 1;
  if (grp * NS >= S) return;  // padding pair (both halves leave)
  const int sl = lane & 15;
  const int seq = grp * NS + sl;
  const bool valid = seq < S;
  const int u0 = 128 * p + 16 * w + 4 * (lane >> 4);  // this lane's 4 units (rows of the gate tiles)

  chunk16 wa[P_NF];  // fragment f = g*8 + kk: rows g*256 + 128p + 16w + (lane&15), k = 32kk + 8(lane>>4) + e
  const chunk16* wsrc = wp + (int64_t)(p * P_NW + w) * P_NF * 64 + lane;
#pragma unroll
  for (int f = 0; f < P_NF; ++f) wa[f] = wsrc[f * 64];
  for (int i = tid; i < NS * 512 / 4; i += 512) ((unsigned*)hb)[i] = 0u;  // h_{-1} = 0 (both halves)

  // exchange slots of this pair: ours [p][parity], the partner's [1-p][parity]; lane tid <-> lane tid
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(xbuf + (int64_t)grp * P_SLOT, (uint32_t)(P_SLOT * 16));
  const uint32_t x_own = (uint32_t)(((p * 2) * 512 + tid) * 16), x_rem = (uint32_t)((((1 - p) * 2) * 512 + tid) * 16);
  const uint32_t tag_base = sync.xtag + 1u;  // tag of step t: tag_base + t; the handshake's: sync.xtag (never 0)

  int ra = 0, rb = -1;
  if (sync.ready) {
    if (sync.time_mode) {
      rb = 0;
    } else {
      const int s_first = grp * NS, s_last = min(S, s_first + NS) - 1;
      while (sync.seq_end[ra] <= s_first) ++ra;
      rb = ra;
      while (sync.seq_end[rb] <= s_last) ++rb;
    }
    if (tid == 0) {  // relaxed poll + one agent acquire (see lstm_resident_kernel)
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      const bool tr = sync.handoff_trace && b == 0;
      if (tr) g_lstm_handoff[0] = g_lstm_handoff[1] = t0;
      for (int r = ra; r <= rb; ++r)
        while (__hip_atomic_load(sync.ready + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < sync.epoch) {
          __builtin_amdgcn_s_sleep(8);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
            if (sync.error) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
        }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tr) g_lstm_handoff[2] = __builtin_amdgcn_s_memrealtime();
    }
  }
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  // gate rows in the pair layout (gx_pair_block): this lane's 16 gate values (4 gates x units u0 .. u0+3)
  // of a step are two 16-byte halves, each wave-load one contiguous KiB (a launch starting mid-group, seq0
  // % 16 != 0, splits it over two blocks; missing sequences read sequence seq0's records)
  const int gs = seq0 + (valid ? seq : 0);
  const bf16* gxs = gx + gx_pair_block(gs >> 4, 0, u0 >> 4, Tn) + (((u0 >> 2) & 3) * 16 + (gs & 15)) * 8;
  const int goff = sync.gx_off;
  auto grow = [&](int t) -> int64_t {  // slot stride of a group: 16 blocks of 1024 elements
    const int r = t + goff;
    return (int64_t)(r >= Tn ? r - Tn : r) * (16 * 1024);
  };
  __syncthreads();  // hb zeroed; ready acquired

  auto hfrag = [&](int kk) -> chunk16 {  // B operand: h[32kk + 8(lane>>4) + e][seq lane&15]
    return *(const chunk16*)(hb + sl * 512 + (((kk * 4 + (lane >> 4)) ^ sl) << 4));
  };
  auto hput = [&](int u, u32x2 v) {  // 4 consecutive units (u % 4 == 0) of sequence sl
    *(u32x2*)(hb + sl * 512 + (((u >> 3) ^ sl) << 4) + (u & 7) * 2) = v;
  };
  const bool samp = ST && blockIdx.x < 8 && tid == 0;
  __shared__ unsigned long long stl[ST ? 20 : 1];  // stamps go to LDS (a global store would join the counted vmcnt)
  auto stamp = [&](int t, int k) {  // diagnostics: g_lstm_stamps[wg][step 100..103][point]
    if constexpr (ST) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long v = __builtin_amdgcn_s_memtime();
      if (samp && t >= sync.stamp_t0 && t < sync.stamp_t0 + 4) stl[(t - sync.stamp_t0) * 5 + k] = v;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int chunk = 0;
  bool dead = false;  // an exchange wait timed out (error word set): the remaining steps do not wait
  // the own / partner k-step ranges index the fragment array: compile-time per half, so the fragments
  // stay in registers (a runtime index would put them in scratch)
  // Every vector-memory op of the step loop is issued by inline asm in a fixed order, and the waits
  // are counted by hand: vmcnt retires in issue order, and the compiler's own accounting falls back to
  // vmcnt(0) at the loop's merge points, which would make each exchange wait also wait for the gx
  // prefetch just issued.  Per step t (steady state):
  //   P  exchange poll (partner's h_{t-1}, t > 0) | G  gx record of step t+2 (2 loads) | R  poll retries
  //   X  exchange publish (h_t)                   | O  h_t row store
  // -> the poll wait is vmcnt(2) (G may stay in flight); gx of step t (issued in step t-2) is waited
  // with vmcnt(7) (at least R X O + P G R X O are younger).  Retries only add younger ops, so both
  // waits stay sufficient.
  const __amdgpu_buffer_rsrc_t orsc =
      make_rsrc(out + (int64_t)grp * NS * out_seq_stride, (uint32_t)((int64_t)min(NS, S - grp * NS) * out_seq_stride * 2));
  const uint32_t o_lane = (uint32_t)(((int64_t)sl * out_seq_stride + u0) * 2);  // lanes of missing sequences: out of range
  auto gload = [&](u32x4 (&gv)[2], int row) {  // gates 0/1 and 2/3 of the lane's 4 units
    const bf16* a = gxs + grow(row);
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(gv[0]) : "v"(a) : "memory");
    asm volatile("global_load_dwordx4 %0, %1, off offset:1024" : "=v"(gv[1]) : "v"(a) : "memory");
  };
  u32x4 ga[2], gb[2];  // gx ring: ga for even steps, gb for odd
  gload(ga, 0);
  gload(gb, Tn > 1 ? 1 : 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // XCD handshake: the exchange stores may stay in the XCD's L2 (default policy instead of
  // write-through: +1.7 % end to end) only when both halves of the pair run on the same XCD, which
  // round-robin placement gives blocks b and b + 8 but nothing guarantees.  Each lane publishes its
  // XCC id in its own parity-1 slot with the tag tag_base - 1 (no step uses it; the slot is first
  // overwritten at step 1, after the partner consumed step 0, i.e. after it read this granule) and
  // reads the partner lane's; a timed-out handshake keeps write-through and sets the error word.
  bool xl2 = sync.xplain > 0;  // VAP_LSTM_XPLAIN: 1 plain stores always, -1 never, 0 (default) by handshake
  if (sync.xplain == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    const uint32_t htag = tag_base - 1u;
    const u32x4 hv = {xcc, htag, xcc, htag};
    asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen sc1\n\ts_nop 2" ::"v"(hv), "v"(x_own + 512u * 16u), "s"(xr)
                 : "memory");
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    u32x4 pv;
    bool ok = true;
    while (true) {
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1\n\ts_waitcnt vmcnt(0)" : "=v"(pv) : "v"(x_rem + 512u * 16u), "s"(xr)
                   : "memory");
      if (__all(pv[1] == htag && pv[3] == htag)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
        if (sync.error && lane == 0) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    xl2 = ok && __all(pv[0] == xcc && pv[2] == xcc);
    if (tid == 0 && b < 64) g_lstm_xcc[b] = xcc | (pv[0] << 8) | ((uint32_t)xl2 << 16) | (1u << 24);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the step loop's hand-counted waits start from zero
  }
  auto run = [&](auto half) {
  constexpr int kown = 4 * decltype(half)::value, krem = 4 - kown;
  auto step = [&](const int t, u32x4 (&gc)[2], u32x4 (&go)[2]) {
    stamp(t, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (t >= 2) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // gc (gx of step t) landed
    stamp(t, 1);
    f32x4 acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const u32x4 q = gc[g >> 1];
      const bf16x4 v = __builtin_bit_cast(bf16x4, (g & 1) ? u32x2{q[2], q[3]} : u32x2{q[0], q[1]});
      acc[g] = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    }
    // the partner's h_{t-1}: issue the poll now, consume it after the own-unit k-steps
    const uint32_t xo_rem = x_rem + (uint32_t)(((t - 1) & 1) * 512 * 16);
    u32x4 xv = {0u, 0u, 0u, 0u};
    if (t > 0) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1" : "=v"(xv) : "v"(xo_rem), "s"(xr) : "memory");
    gload(gc, t + 2 < Tn ? t + 2 : Tn - 1);  // gx of step t+2 into the slot just consumed
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const chunk16 hf = hfrag(kown + q);
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = mfma_chunk<bf16>(wa[g * 8 + kown + q], hf, acc[g]);
    }
    stamp(t, 2);
    if (t > 0) {
      __builtin_amdgcn_sched_barrier(0);  // the own-unit MFMAs stay ahead of the wait
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // P landed (G may still be in flight)
      const uint32_t want = tag_base + (uint32_t)(t - 1);
      uint64_t t0 = 0;
      while (!dead && !__all(xv[1] == want && xv[3] == want)) {
        if (!t0) {
          t0 = __builtin_amdgcn_s_memrealtime();
        } else if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
          if (sync.error && lane == 0) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          dead = true;  // the partner is gone: no further waits (the launch drains in microseconds)
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1\n\ts_waitcnt vmcnt(0)" : "=v"(xv) : "v"(xo_rem), "s"(xr)
                     : "memory");
      }
      hput(u0 ^ 128, u32x2{xv[0], xv[2]});  // the partner lane's units: 128(1-p) + 16w + 4(lane>>4)
    }
    stamp(t, 3);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // B1: the partner's half of h_{t-1} is in the image
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const chunk16 hf = hfrag(krem + q);
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = mfma_chunk<bf16>(wa[g * 8 + krem + q], hf, acc[g]);
    }
    float hv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) lstm_cell<PRE>(acc, r, c[r], hv[r]);
    const u32x2 hp = pack_bf16x4(hv[0], hv[1], hv[2], hv[3]);
    const uint32_t tag = tag_base + (uint32_t)t;
    const u32x4 xo = {hp[0], tag, hp[1], tag};
    const uint32_t xoff = x_own + (uint32_t)((t & 1) * 512 * 16);
    if (xl2)  // both halves on one XCD (handshake above): the exchange stays in that XCD's L2
      asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 2" ::"v"(xo), "v"(xoff), "s"(xr) : "memory");
    else  // publish to the partner (write-through)
      asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen sc1\n\ts_nop 2" ::"v"(xo), "v"(xoff), "s"(xr) : "memory");
    // (the s_nops: a VALU write of a store's data VGPRs right after a dwordx3/x4 store is a hazard the
    // compiler does not see through inline asm)
    asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen\n\ts_nop 2" ::"v"(hp), "v"(o_lane + (uint32_t)t * (HD * 2)),
                 "s"(orsc) : "memory");
    hput(u0, hp);  // own units of h_t (the own-unit reads of this step retired before B1)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // B2: own h_t visible to every wave
    stamp(t, 4);
    if (sync.time_mode && chunk < sync.nr && t + 1 >= sync.seq_end[chunk]) {
      // end of a time chunk: publish its h rows, then wait for the next chunk's gate projection
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int c0 = chunk;
      while (chunk < sync.nr && t + 1 >= sync.seq_end[chunk]) ++chunk;
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int cc = c0; cc < chunk; ++cc)
          __hip_atomic_fetch_add(sync.done + cc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool tr = sync.handoff_trace && b == 0;
        if (tr) g_lstm_handoff[3 + 3 * c0] = __builtin_amdgcn_s_memrealtime();
        if (chunk < sync.nr) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          if (tr) g_lstm_handoff[1 + 3 * chunk] = t0;
          while (__hip_atomic_load(sync.ready + chunk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < sync.epoch) {
            __builtin_amdgcn_s_sleep(8);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
              if (sync.error) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              break;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (tr) g_lstm_handoff[2 + 3 * chunk] = __builtin_amdgcn_s_memrealtime();
        }
      }
      if (chunk < sync.nr) {  // rows t+1 and t+2 may have been prefetched before the hand-off: reload
        __syncthreads();
        gload(go, t + 1);
        gload(gc, t + 2 < Tn ? t + 2 : Tn - 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
  };
  for (int t = 0; t < Tn; t += 2) {
    step(t, ga, gb);
    if (t + 1 < Tn) step(t + 1, gb, ga);
  }  };
  if (p == 0) run(std::integral_constant<int, 0>{});
  else run(std::integral_constant<int, 1>{});
  if constexpr (ST) {
    if (samp && Tn >= sync.stamp_t0 + 4)
      for (int i = 0; i < 20; ++i) g_lstm_stamps[blockIdx.x][i / 5][i % 5] = stl[i];
  }
  if (sync.ready && !sync.time_mode) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int r = ra; r <= rb; ++r) __hip_atomic_fetch_add(sync.done + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}


// ------------------------------------------------------------------------------------------
// bf16 perf mode, W_hh split over a QUAD of workgroups (VAP_LSTM_QUAD): four CUs per 16 sequences.
//
// The pair kernel spends ~1k cycles of MFMA and ~1k of cell update per SIMD and step (two waves per
// SIMD in the same phase).  Here quarter q of a quad owns hidden units [64q, 64q + 64): 4 gates x 64
// units = 256 W_hh rows = 128 KiB bf16 in registers across 4 waves (one per SIMD, 32 fragments each;
// wave w owns units 64q + 16w .. +16, one row tile per gate), so per SIMD and step the matrix work
// and the cell update both halve (32 MFMAs and 4 cells per lane) at the price of three exchange
// partners instead of one.  Same operands as the pair kernel: the pair-packed W_hh (pair half p,
// wave w' is quarter 2p + w'/4, wave w' % 4) and the pair-layout gate rows (a lane's 16-unit block
// is 4q + w, the same records).  Exchange as lstm_pair_kernel with three partners: one 16-byte
// {2 x bf16, tag} x 2 granule per lane and step into the quad's slot [quarter][parity][tid], polled
// by the same lane of each partner (sc1 loads) and issued before the own-unit k-steps (2 of 8).  The
// XCC handshake covers the whole quad (plain stores only when all four quarters share an XCD).
// Quads are blocks (b, b+8, b+16, b+24) of each 32-block group; every spin is bounded.
// ------------------------------------------------------------------------------------------
constexpr int QB_NW = 4, QB_NF = 32;            // waves per workgroup, W fragments per wave
constexpr int QB_SLOT = 4 * 2 * 256;            // 16-byte exchange slots per quad: [quarter][parity][tid]
static_assert(QB_SLOT == P_SLOT, "the quad and pair kernels share the exchange buffer sizing");

template <bool ST>
__global__ __launch_bounds__(256, 1) void lstm_quadb_kernel(const bf16* __restrict__ gx, int seq0, int S, int Tn,
                                                            const chunk16* __restrict__ wp, bf16* __restrict__ out,
                                                            int64_t out_seq_stride, LstmSync sync, u32x4* xbuf) {
  __shared__ __attribute__((aligned(16))) unsigned char hb[NS * 512];  // h_{t-1} [seq][256], chunk ^= seq
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x;
  const int grp = (b >> 5) * 8 + (b & 7), q = (b >> 3) & 3;
  if (grp * NS >= S) return;  // padding quad (all four quarters leave)
  const int sl = lane & 15;
  const int seq = grp * NS + sl;
  const bool valid = seq < S;
  const int u0 = 64 * q + 16 * w + 4 * (lane >> 4);  // this lane's 4 units

  chunk16 wa[QB_NF];  // fragment f = g*8 + kk: rows g*256 + 64q + 16w + (lane&15), k = 32kk + 8(lane>>4) + e
  const chunk16* wsrc = wp + (int64_t)(q * QB_NW + w) * QB_NF * 64 + lane;  // pair packing, (p, w') = (q/2, 4(q%2) + w)
#pragma unroll
  for (int f = 0; f < QB_NF; ++f) wa[f] = wsrc[f * 64];
  for (int i = tid; i < NS * 512 / 4; i += 256) ((unsigned*)hb)[i] = 0u;  // h_{-1} = 0

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(xbuf + (int64_t)grp * QB_SLOT, (uint32_t)(QB_SLOT * 16));
  auto xoff = [&](int qq, int par) -> uint32_t { return (uint32_t)(((qq * 2 + par) * 256 + tid) * 16); };
  const uint32_t tag_base = sync.xtag + 1u;  // tag of step t: tag_base + t; the handshake's: sync.xtag (never 0)

  int ra = 0, rb = -1;
  if (sync.ready) {
    if (sync.time_mode) {
      rb = 0;
    } else {
      const int s_first = grp * NS, s_last = min(S, s_first + NS) - 1;
      while (sync.seq_end[ra] <= s_first) ++ra;
      rb = ra;
      while (sync.seq_end[rb] <= s_last) ++rb;
    }
    if (tid == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (int r = ra; r <= rb; ++r)
        while (__hip_atomic_load(sync.ready + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < sync.epoch) {
          __builtin_amdgcn_s_sleep(8);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
            if (sync.error) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
        }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  const int gs = seq0 + (valid ? seq : 0);
  const bf16* gxs = gx + gx_pair_block(gs >> 4, 0, u0 >> 4, Tn) + (((u0 >> 2) & 3) * 16 + (gs & 15)) * 8;
  const int goff = sync.gx_off;
  auto grow = [&](int t) -> int64_t {
    const int r = t + goff;
    return (int64_t)(r >= Tn ? r - Tn : r) * (16 * 1024);
  };
  // Every vector-memory op of the step loop is inline asm in a fixed order with hand-counted waits (as
  // lstm_pair_kernel; the compiler's own accounting falls back to vmcnt(0) at the loop's merge points,
  // which would make the gx wait also wait for the polls just issued).  Per step t (steady state):
  //   P  3 exchange polls (partners' h_{t-1}, t > 0) | G  gx record of step t+2 (2 loads) | R  retries
  //   X  exchange publish (h_t)                        | O  h_t row store
  // -> the poll wait is vmcnt(2) (G may stay in flight); gx of step t (issued in step t-2) is waited with
  // vmcnt(9) (X O of step t-2 and P G X O of step t-1 are younger).  Retries only add younger ops.
  auto gload = [&](u32x4 (&gv)[2], int row) {  // gates 0/1 and 2/3 of the lane's 4 units
    const bf16* a = gxs + grow(row);
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(gv[0]) : "v"(a) : "memory");
    asm volatile("global_load_dwordx4 %0, %1, off offset:1024" : "=v"(gv[1]) : "v"(a) : "memory");
  };
  auto poll = [&](u32x4& v, uint32_t off) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1" : "=v"(v) : "v"(off), "s"(xr) : "memory");
  };
  __syncthreads();  // hb zeroed; ready acquired

  auto hfrag = [&](int kk) -> chunk16 {
    return *(const chunk16*)(hb + sl * 512 + (((kk * 4 + (lane >> 4)) ^ sl) << 4));
  };
  auto hput = [&](int u, u32x2 v) { *(u32x2*)(hb + sl * 512 + (((u >> 3) ^ sl) << 4) + (u & 7) * 2) = v; };
  const bool samp = ST && blockIdx.x < 8 && tid == 0;
  __shared__ unsigned long long stl[ST ? 20 : 1];
  auto stamp = [&](int t, int k) {
    if constexpr (ST) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long v = __builtin_amdgcn_s_memtime();
      if (samp && t >= sync.stamp_t0 && t < sync.stamp_t0 + 4) stl[(t - sync.stamp_t0) * 5 + k] = v;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  const __amdgpu_buffer_rsrc_t orsc =
      make_rsrc(out + (int64_t)grp * NS * out_seq_stride, (uint32_t)((int64_t)min(NS, S - grp * NS) * out_seq_stride * 2));
  const uint32_t o_lane = (uint32_t)(((int64_t)sl * out_seq_stride + u0) * 2);  // missing sequences: out of range

  // XCC handshake over the quad (see lstm_pair_kernel): plain exchange stores only when all four
  // quarters run on one XCD; the parity-1 slots carry the ids under a tag no step uses.
  bool xl2 = sync.xplain > 0;
  if (sync.xplain == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    const uint32_t htag = tag_base - 1u;
    buf_store16_wt(xr, xoff(q, 1), u32x4{xcc, htag, xcc, htag});
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true, same = true;
    for (int p = 1; p < 4 && ok; ++p) {
      while (true) {
        const u32x4 pv = xload(xr, xoff((q + p) & 3, 1));
        if (__all(pv[1] == htag && pv[3] == htag)) {
          same = same && __all(pv[0] == xcc && pv[2] == xcc);
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
          if (sync.error && lane == 0) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    xl2 = ok && same;
    if (tid == 0 && b < 64) g_lstm_xcc[b] = xcc | ((uint32_t)xl2 << 16) | (1u << 24);
  }
  u32x4 ga[2], gb[2];  // gx ring: ga for even steps, gb for odd
  gload(ga, 0);
  gload(gb, Tn > 1 ? 1 : 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the step loop's hand-counted waits start from zero
  // settle the W fragment loads in the compiler's own bookkeeping here (an asm use makes it wait for
  // them): left pending, it re-waits for them inside the step loop with counts that include the loop's
  // hand-issued polls and gx loads
#pragma unroll
  for (int f = 0; f < QB_NF; ++f) asm volatile("" ::"v"(wa[f]));
  int chunk = 0;
  bool dead = false;
  auto run = [&](auto qc) {
    constexpr int Q = decltype(qc)::value;
    auto kstep = [&](f32x4 (&acc)[4], int kk) {
      const chunk16 hf = hfrag(kk);
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = mfma_chunk<bf16>(wa[g * 8 + kk], hf, acc[g]);
    };
    auto step = [&](const int t, u32x4 (&gc)[2], u32x4 (&go)[2]) {
      stamp(t, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (t >= 2) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");  // gc (gx of step t) landed
      f32x4 acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u32x4 v4 = gc[g >> 1];
        const bf16x4 v = __builtin_bit_cast(bf16x4, (g & 1) ? u32x2{v4[2], v4[3]} : u32x2{v4[0], v4[1]});
        acc[g] = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
      }
      stamp(t, 1);
      const int par = (t - 1) & 1;
      u32x4 xv[3];
      if (t > 0) {
#pragma unroll
        for (int p = 0; p < 3; ++p) poll(xv[p], xoff((Q + 1 + p) & 3, par));
      }
      gload(gc, t + 2 < Tn ? t + 2 : Tn - 1);  // gx of step t+2 into the slot just consumed
      kstep(acc, 2 * Q);
      kstep(acc, 2 * Q + 1);
      stamp(t, 2);
      if (t > 0) {
        __builtin_amdgcn_sched_barrier(0);  // the own-unit MFMAs stay ahead of the waits
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // P landed (G may still be in flight)
        const uint32_t want = tag_base + (uint32_t)(t - 1);
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          uint64_t t0 = 0;
          while (!dead && !__all(xv[p][1] == want && xv[p][3] == want)) {
            if (!t0) {
              t0 = __builtin_amdgcn_s_memrealtime();
            } else if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
              if (sync.error && lane == 0) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              dead = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1\n\ts_waitcnt vmcnt(0)" : "=v"(xv[p])
                         : "v"(xoff((Q + 1 + p) & 3, par)), "s"(xr) : "memory");
          }
          hput(64 * ((Q + 1 + p) & 3) + 16 * w + 4 * (lane >> 4), u32x2{xv[p][0], xv[p][2]});
        }
      }
      stamp(t, 3);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B1: the partners' units of h_{t-1}
      if constexpr (Q != 0) { kstep(acc, 0); kstep(acc, 1); }
      if constexpr (Q != 1) { kstep(acc, 2); kstep(acc, 3); }
      if constexpr (Q != 2) { kstep(acc, 4); kstep(acc, 5); }
      if constexpr (Q != 3) { kstep(acc, 6); kstep(acc, 7); }
      float hv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) lstm_cell<true>(acc, r, c[r], hv[r]);
      const u32x2 hp = pack_bf16x4(hv[0], hv[1], hv[2], hv[3]);
      const uint32_t tag = tag_base + (uint32_t)t;
      const u32x4 xo = {hp[0], tag, hp[1], tag};
      // (the s_nops: a VALU write of a store's data VGPRs right after a dwordx3/x4 store is a hazard the
      // compiler does not see through inline asm)
      if (xl2)  // the whole quad on one XCD: the exchange stays in that XCD's L2
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 2" ::"v"(xo), "v"(xoff(Q, t & 1)), "s"(xr)
                     : "memory");
      else  // write-through
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen sc1\n\ts_nop 2" ::"v"(xo), "v"(xoff(Q, t & 1)), "s"(xr)
                     : "memory");
      asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen\n\ts_nop 2" ::"v"(hp), "v"(o_lane + (uint32_t)t * (HD * 2)),
                   "s"(orsc) : "memory");
      hput(u0, hp);  // own units of h_t (the own-unit reads of this step retired before B1)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B2: own h_t visible to every wave
      stamp(t, 4);
      if (sync.time_mode && chunk < sync.nr && t + 1 >= sync.seq_end[chunk]) {
        // end of a time chunk: publish its h rows, then wait for the next chunk's gate projection
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int c0 = chunk;
        while (chunk < sync.nr && t + 1 >= sync.seq_end[chunk]) ++chunk;
        if (tid == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          for (int cc = c0; cc < chunk; ++cc)
            __hip_atomic_fetch_add(sync.done + cc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (chunk < sync.nr) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(sync.ready + chunk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < sync.epoch) {
              __builtin_amdgcn_s_sleep(8);
              if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
                if (sync.error) __hip_atomic_store(sync.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
              }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        }
        if (chunk < sync.nr) {  // rows t+1 and t+2 may have been prefetched before the hand-off: reload
          __syncthreads();
          gload(go, t + 1 < Tn ? t + 1 : Tn - 1);
          gload(gc, t + 2 < Tn ? t + 2 : Tn - 1);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
    };
    for (int t = 0; t < Tn; t += 2) {
      step(t, ga, gb);
      if (t + 1 < Tn) step(t + 1, gb, ga);
    }
  };
  switch (q) {
    case 0: run(std::integral_constant<int, 0>{}); break;
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    default: run(std::integral_constant<int, 3>{}); break;
  }
  if constexpr (ST) {
    if (samp && Tn >= sync.stamp_t0 + 4)
      for (int i = 0; i < 20; ++i) g_lstm_stamps[blockIdx.x][i / 5][i % 5] = stl[i];
  }
  if (sync.ready && !sync.time_mode) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int r = ra; r <= rb; ++r) __hip_atomic_fetch_add(sync.done + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}


// ------------------------------------------------------------------------------------------
// fp32 parity mode: W_hh split over a QUAD of workgroups, products on split-bf16 operands.
//
// The fp32 recurrence on v_mfma_f32_16x16x4_f32 (lstm_kernel<float>) streams W_hh from L2 at one CU
// per 16 sequences: 1024 MFMAs of 32 cycles per wave and step (~13.6 us of issue, 19 us per step).
// Here both operands are fp32 values carried as hi + lo bf16 pairs (hi = bf16(x), lo = bf16(x - hi))
// and every product as hi_w hi_h + hi_w lo_h + lo_w hi_h, three v_mfma_f32_16x16x32_bf16 with fp32
// accumulation (the lo lo term is ~2^-18 of the product; the gate pre-activations stay within ~1e-6 of
// fp32).  Workgroup q of a quad owns hidden units [64q, 64q + 64): 4 gates x 64 units = 256 W_hh rows,
// hi + lo = 256 KiB, held in registers by 4 waves (one per SIMD, 64 fragments = 256 VGPRs each); wave w
// owns units 64q + 16w .. +16 (one row tile per gate: 96 MFMAs and 4 cells per lane per step, ~1.5k
// cycles of matrix issue).  The cell update runs in fp32 (v_exp / v_rcp forms, abs. error ~2e-7, as
// lstm_kernel<float>); c and h stay fp32 and h_t rows are stored fp32.
// Exchange (as lstm_pair_kernel, with three partners): every lane publishes its 4 fp32 h values as four
// 8-byte {h, tag} granules in two 16-byte write-through stores into the quad's slot for step parity t&1;
// the same lane of each partner polls those slots (sc1 loads) until every tag matches, then writes the
// values, split into hi / lo, into its two LDS images of h.  The polls are issued before the own-unit
// k-steps (2 of 8), so their latency overlaps those MFMAs.  Two parity slots suffice (a quarter writes
// h_t only after reading every partner's h_{t-1}, published after they read our h_{t-2}).  Quads are
// blocks (b, b+8, b+16, b+24) of each 32-block group (one XCD under round-robin placement: speed only);
// every spin is bounded (~2 s, then the error word is set and the launch runs on without waiting).
// ------------------------------------------------------------------------------------------
constexpr int Q_NW = 4, Q_NF = 64;              // waves per workgroup, fragments per wave (4 g x 8 kk x hi/lo)
constexpr int Q_SLOT = 4 * 2 * 256 * 2;         // 16-byte exchange slots per quad: [quarter][parity][tid][2]

template <int Q>
VAP_DEV void quad_steps(const float* __restrict__ gxs, int Tn, int S, const chunk16 (&wf)[Q_NF], unsigned char* hh,
                        unsigned char* hl, __amdgpu_buffer_rsrc_t xr, __amdgpu_buffer_rsrc_t orsc, uint32_t o_lane,
                        uint32_t tag_base, unsigned* err, int tid) {
  const int lane = tid & 63, w = tid >> 6, sl = lane & 15;
  const int u0 = 64 * Q + 16 * w + 4 * (lane >> 4);
  auto hfrag = [&](const unsigned char* img, int kk) -> chunk16 {  // h[32kk + 8(lane>>4) + e][seq sl]
    return *(const chunk16*)(img + sl * 512 + (((kk * 4 + (lane >> 4)) ^ sl) << 4));
  };
  auto hput = [&](int u, float a, float b, float c, float d) {  // units u .. u+3 of sequence sl, split
    const bf16x4 hi = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
    const bf16x4 lo = {(bf16)(a - (float)hi[0]), (bf16)(b - (float)hi[1]), (bf16)(c - (float)hi[2]),
                       (bf16)(d - (float)hi[3])};
    const int off = sl * 512 + (((u >> 3) ^ sl) << 4) + (u & 7) * 2;
    *(bf16x4*)(hh + off) = hi;
    *(bf16x4*)(hl + off) = lo;
  };
  // exchange slot byte offsets: quarter qq, parity par, this thread, granule pair j
  auto xoff = [&](int qq, int par, int j) -> uint32_t { return (uint32_t)((((qq * 2 + par) * 256 + tid) * 2 + j) * 16); };
  // gates of step t: 4 x 16 B (gate g at column g*256 + u0), two steps ahead (compiler-tracked loads: the
  // waits are the compiler's, so no register of an in-flight load is ever read early)
  auto gload = [&](u32x4 (&gv)[4], int t) {
    const float* a = gxs + (int64_t)t * 1024;
#pragma unroll
    for (int g = 0; g < 4; ++g) gv[g] = *(const u32x4*)(a + g * 256);
  };
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  u32x4 ga[4], gb[4];
  gload(ga, 0);
  gload(gb, Tn > 1 ? 1 : 0);
  bool dead = false;
  // the weight fragments stay in AGPRs as the MFMAs' A operand (inline asm, mfma_a): LEAD pads the
  // VALU-write -> srcC wait of a fresh accumulator, TAIL the MFMA -> VALU wait after the step's last one
  constexpr int KLAST = Q == 3 ? 5 : 7;
  auto kstep = [&](f32x4 (&acc)[4], auto kkc) {
    constexpr int kk = decltype(kkc)::value;
    constexpr int LEAD = kk == 2 * Q ? 1 : 0, TAIL = kk == KLAST ? 1 : 0;
    const chunk16 bh = hfrag(hh, kk), bl = hfrag(hl, kk);
#pragma unroll
    for (int g = 0; g < 4; ++g) mfma_a<LEAD, 0>(acc[g], wf[(g * 8 + kk) * 2 + 1], bh);  // lo_w hi_h
#pragma unroll
    for (int g = 0; g < 4; ++g) mfma_a<0, 0>(acc[g], wf[(g * 8 + kk) * 2], bl);        // hi_w lo_h
    mfma_a<0, 0>(acc[0], wf[(0 * 8 + kk) * 2], bh);                                      // hi_w hi_h
    mfma_a<0, 0>(acc[1], wf[(1 * 8 + kk) * 2], bh);
    mfma_a<0, 0>(acc[2], wf[(2 * 8 + kk) * 2], bh);
    mfma_a<0, TAIL>(acc[3], wf[(3 * 8 + kk) * 2], bh);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I5 = std::integral_constant<int, 5>;
  using I6 = std::integral_constant<int, 6>;
  using I7 = std::integral_constant<int, 7>;
  auto step = [&](const int t, u32x4 (&gc)[4]) {
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = __builtin_bit_cast(f32x4, gc[g]);
    u32x4 xv[3][2];
    const int par = (t - 1) & 1;
    if (t > 0) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j) xv[p][j] = xload(xr, xoff((Q + 1 + p) & 3, par, j));
    }
    gload(gc, t + 2 < Tn ? t + 2 : Tn - 1);  // gates of step t+2 into the slot just consumed
    kstep(acc, std::integral_constant<int, 2 * Q>{});
    kstep(acc, std::integral_constant<int, 2 * Q + 1>{});
    if (t > 0) {
      __builtin_amdgcn_sched_barrier(0);  // the own-unit MFMAs stay ahead of the wait
      const uint32_t want = tag_base + (uint32_t)(t - 1);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        uint64_t t0 = 0;
        while (!dead && !__all(xv[p][0][1] == want && xv[p][0][3] == want && xv[p][1][1] == want && xv[p][1][3] == want)) {
          if (!t0) {
            t0 = __builtin_amdgcn_s_memrealtime();
          } else if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
            if (err && lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            dead = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          xv[p][0] = xload(xr, xoff((Q + 1 + p) & 3, par, 0));
          xv[p][1] = xload(xr, xoff((Q + 1 + p) & 3, par, 1));
        }
        const int uq = 64 * ((Q + 1 + p) & 3) + 16 * w + 4 * (lane >> 4);  // the partner lane's units
        // (bit-cast whole vectors: hipcc lowers __builtin_bit_cast(float, v[i]) of an ext_vector element to
        // element 0 whatever i is, vap_common.h)
        const f32x4 v0 = __builtin_bit_cast(f32x4, xv[p][0]), v1 = __builtin_bit_cast(f32x4, xv[p][1]);
        hput(uq, v0[0], v0[2], v1[0], v1[2]);
      }
    }
    // (barriers as asm with a memory clobber: the s_barrier builtin does not order the LDS reads after it)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B1: the partners' units of h_{t-1} are in
                                                                     // the images
    if constexpr (Q != 0) { kstep(acc, I0{}); kstep(acc, I1{}); }
    if constexpr (Q != 1) { kstep(acc, I2{}); kstep(acc, I3{}); }
    if constexpr (Q != 2) { kstep(acc, I4{}); kstep(acc, I5{}); }
    if constexpr (Q != 3) { kstep(acc, I6{}); kstep(acc, I7{}); }
    __builtin_amdgcn_sched_barrier(0);  // the cell's VALU reads stay behind the TAIL wait
    float hv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ig = cell_sig(acc[0][r]), fg = cell_sig(acc[1][r]), gg = cell_tanh(acc[2][r]), og = cell_sig(acc[3][r]);
      c[r] = fg * c[r] + ig * gg;
      hv[r] = og * cell_tanh(c[r]);
    }
    const uint32_t tag = tag_base + (uint32_t)t;
    const u32x4 x0 = {__builtin_bit_cast(uint32_t, hv[0]), tag, __builtin_bit_cast(uint32_t, hv[1]), tag};
    const u32x4 x1 = {__builtin_bit_cast(uint32_t, hv[2]), tag, __builtin_bit_cast(uint32_t, hv[3]), tag};
    const u32x4 hrow = {__builtin_bit_cast(uint32_t, hv[0]), __builtin_bit_cast(uint32_t, hv[1]),
                        __builtin_bit_cast(uint32_t, hv[2]), __builtin_bit_cast(uint32_t, hv[3])};
    buf_store16_wt(xr, xoff(Q, t & 1, 0), x0);  // write-through (sc1): the partners poll with sc1 loads
    buf_store16_wt(xr, xoff(Q, t & 1, 1), x1);
    buf_store16(orsc, o_lane + (uint32_t)t * (HD * 4), hrow);
    hput(u0, hv[0], hv[1], hv[2], hv[3]);  // own units of h_t (this step's own-unit reads retired before B1)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B2: own h_t visible to every wave
  };
  for (int t = 0; t < Tn; t += 2) {
    step(t, ga);
    if (t + 1 < Tn) step(t + 1, gb);
  }
}

__global__ __launch_bounds__(256, 1) void lstm_quad_kernel(const float* __restrict__ gx, int S, int Tn,
                                                           const chunk16* __restrict__ wp, float* __restrict__ out,
                                                           int64_t out_seq_stride, u32x4* xbuf, unsigned xtag,
                                                           unsigned* err) {
  __shared__ __attribute__((aligned(16))) unsigned char hh[NS * 512];  // h_{t-1} hi [seq][256] bf16, chunk ^= seq
  __shared__ __attribute__((aligned(16))) unsigned char hl[NS * 512];  // h_{t-1} lo
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x;
  const int grp = (b >> 5) * 8 + (b & 7), q = (b >> 3) & 3;
  if (grp * NS >= S) return;  // padding quad (all four quarters leave)
  const int sl = lane & 15;
  const int seq = grp * NS + sl;
  const bool valid = seq < S;
  const int u0 = 64 * q + 16 * w + 4 * (lane >> 4);

  chunk16 wf[Q_NF];  // fragment (g*8 + kk)*2 + s: rows g*256 + 64q + 16w + (lane&15), k = 32kk + 8(lane>>4) + e
  const chunk16* wsrc = wp + (int64_t)(q * Q_NW + w) * Q_NF * 64 + lane;
#pragma unroll
  for (int f = 0; f < Q_NF; ++f) wf[f] = wsrc[f * 64];
  for (int i = tid; i < NS * 512 / 4; i += 256) {
    ((unsigned*)hh)[i] = 0u;  // h_{-1} = 0
    ((unsigned*)hl)[i] = 0u;
  }
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(xbuf + (int64_t)grp * Q_SLOT, (uint32_t)(Q_SLOT * 16));
  const __amdgpu_buffer_rsrc_t orsc =
      make_rsrc(out + (int64_t)grp * NS * out_seq_stride, (uint32_t)((int64_t)min(NS, S - grp * NS) * out_seq_stride * 4));
  const uint32_t o_lane = (uint32_t)(((int64_t)sl * out_seq_stride + u0) * 4);  // missing sequences: out of range
  const float* gxs = gx + (int64_t)(valid ? seq : grp * NS) * Tn * 1024 + u0;
  __syncthreads();
  const uint32_t tag_base = xtag;  // tag of step t: xtag + t
  switch (q) {
    case 0: quad_steps<0>(gxs, Tn, S, wf, hh, hl, xr, orsc, o_lane, tag_base, err, tid); break;
    case 1: quad_steps<1>(gxs, Tn, S, wf, hh, hl, xr, orsc, o_lane, tag_base, err, tid); break;
    case 2: quad_steps<2>(gxs, Tn, S, wf, hh, hl, xr, orsc, o_lane, tag_base, err, tid); break;
    default: quad_steps<3>(gxs, Tn, S, wf, hh, hl, xr, orsc, o_lane, tag_base, err, tid); break;
  }
}

// quad layout: Wq[q][w][f = (g*8 + kk)*2 + s][lane][e] = split_s(W[g*256 + 64q + 16w + (l&15)][32kk + 8(l>>4) + e])
__global__ void pack_whh_quad_kernel(const float* __restrict__ whh, bf16* __restrict__ out) {
  const int64_t n = (int64_t)G4 * HD * 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7);
    const int l = (int)((i >> 3) & 63);
    const int f = (int)((i >> 9) & 63);
    const int w = (int)((i >> 15) & 3);
    const int q = (int)(i >> 17);
    const int sp = f & 1, kk = (f >> 1) & 7, g = f >> 4;
    const int row = g * HD + 64 * q + 16 * w + (l & 15);
    const int k = 32 * kk + 8 * (l >> 4) + e;
    const float x = whh[(int64_t)row * HD + k];
    const bf16 hi = (bf16)x;
    out[i] = sp ? (bf16)(x - (float)hi) : hi;
  }
}

// Wp[w][f = rt*8 + kg][lane][e] = W[g*256 + 64w + 16ut + (l&15)][32kg + 8(l>>4) + e],  rt = g*4 + ut
// gate-row scale of the pre-scaled packing (lstm_cell<true>): -log2e on i / f / o, 2 log2e on g
VAP_DEV float gate_scale(int row) { return (row >> 8) == 2 ? KC : -0.5f * KC; }

__global__ void pack_whh_resident_kernel(const float* __restrict__ whh, bf16* __restrict__ out, int pre) {
  const int64_t n = (int64_t)G4 * HD;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7);
    const int l = (int)((i >> 3) & 63);
    const int f = (int)((i >> 9) & 127);
    const int w = (int)(i >> 16);
    const int rt = f >> 3, kg = f & 7, g = rt >> 2, ut = rt & 3;
    const int row = g * HD + 64 * w + 16 * ut + (l & 15);
    const int k = 32 * kg + 8 * (l >> 4) + e;
    out[i] = (bf16)(whh[(int64_t)row * HD + k] * (pre ? gate_scale(row) : 1.0f));
  }
}

// pair layout: Wp[p][w][f = g*8 + kk][lane][e] = W[g*256 + 128p + 16w + (l&15)][32kk + 8(l>>4) + e]
__global__ void pack_whh_pair_kernel(const float* __restrict__ whh, bf16* __restrict__ out, int pre) {
  const int64_t n = (int64_t)G4 * HD;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7);
    const int l = (int)((i >> 3) & 63);
    const int f = (int)((i >> 9) & 31);
    const int w = (int)((i >> 14) & 7);
    const int p = (int)(i >> 17);
    const int g = f >> 3, kk = f & 7;
    const int row = g * HD + 128 * p + 16 * w + (l & 15);
    const int k = 32 * kk + 8 * (l >> 4) + e;
    out[i] = (bf16)(whh[(int64_t)row * HD + k] * (pre ? gate_scale(row) : 1.0f));
  }
}

// W_ih [1024][256] fp32 -> bf16 with the gate-row scales and the rows in the gx_wrow order of the c_pair
// gate projection (its lanes then hold whole records of the pair layout); b = (b_ih + b_hh) * scale,
// permuted alike
__global__ void pack_wih_prescaled_kernel(const float* __restrict__ wih, bf16* __restrict__ out,
                                          const float* __restrict__ bih, const float* __restrict__ bhh,
                                          float* __restrict__ b) {
  const int64_t n = (int64_t)G4 * HD;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(i / HD), k = (int)(i % HD);
    const int col = gx_wrow(row >> 8, row & 255);
    out[(int64_t)col * HD + k] = (bf16)(wih[i] * gate_scale(row));
    if (i < G4) b[gx_wrow((int)i >> 8, (int)i & 255)] = (bih[i] + bhh[i]) * gate_scale((int)i);
  }
}

// [S][Tn][1024] gate rows in the natural order -> the pair layout (kernel tests)
__global__ void pack_gx_pair_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, int S, int Tn) {
  const int64_t n = (int64_t)S * Tn * G4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int col = (int)(i & (G4 - 1));
    const int64_t r = i >> 10;
    out[gx_pair_off((int)(r / Tn), (int)(r % Tn), col >> 8, col & 255, Tn)] = in[i];
  }
}

__global__ void scale_gates_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (bf16)((float)in[i] * gate_scale((int)(i & (G4 - 1))));
}

}  // namespace

hipError_t launch_pack_gx_pair(const bf16* in, bf16* out, int S, int Tn, hipStream_t st) {
  hipLaunchKernelGGL(pack_gx_pair_kernel, dim3(1024), dim3(256), 0, st, in, out, S, Tn);
  return hipGetLastError();
}

// gx rows [.][1024] -> the pre-scaled gate units of lstm_cell<true> (kernel tests)
hipError_t launch_scale_gates(const bf16* in, bf16* out, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(scale_gates_kernel, dim3(1024), dim3(256), 0, st, in, out, n);
  return hipGetLastError();
}

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

hipError_t launch_lstm_resident(const bf16* gx, int S, int Tn, const bf16* whh_packed, bf16* out,
                                int64_t out_seq_stride, hipStream_t st, const LstmSync* sync, bool prescaled) {
  if (S <= 0 || Tn <= 0) return hipErrorInvalidValue;
  LstmSync sy{};
  if (sync) {
    if (sync->nr < 1 || sync->nr > 16 || sync->seq_end[sync->nr - 1] < (sync->time_mode ? Tn : S))
      return hipErrorInvalidValue;
    for (int c = 1; c < sync->nr; ++c)
      if (sync->seq_end[c] <= sync->seq_end[c - 1]) return hipErrorInvalidValue;
    if (sync->gx_off < 0 || sync->gx_off >= Tn) return hipErrorInvalidValue;
    sy = *sync;
  }
  static const bool stamps = getenv("VAP_LSTM_STAMPS") != nullptr;
  const dim3 grid((S + NS - 1) / NS);
  const chunk16* wpk = (const chunk16*)whh_packed;
  if (stamps && prescaled) hipLaunchKernelGGL((lstm_resident_kernel<true, true>), grid, dim3(256), 0, st, gx, S, Tn, wpk, out, out_seq_stride, sy);
  else if (stamps) hipLaunchKernelGGL((lstm_resident_kernel<true, false>), grid, dim3(256), 0, st, gx, S, Tn, wpk, out, out_seq_stride, sy);
  else if (prescaled) hipLaunchKernelGGL((lstm_resident_kernel<false, true>), grid, dim3(256), 0, st, gx, S, Tn, wpk, out, out_seq_stride, sy);
  else hipLaunchKernelGGL((lstm_resident_kernel<false, false>), grid, dim3(256), 0, st, gx, S, Tn, wpk, out, out_seq_stride, sy);
  return hipGetLastError();
}
size_t lstm_pair_xbuf_bytes(int S) { return (size_t)((S + NS - 1) / NS) * P_SLOT * 16; }
int lstm_pair_workgroups(int S, int quad) { return (quad ? 4 : 2) * ((S + NS - 1) / NS); }

hipError_t launch_lstm_pair(const bf16* gx, int seq0, int S, int Tn, const bf16* whh_pair, bf16* out,
                            int64_t out_seq_stride, hipStream_t st, const LstmSync* sync, void* xbuf, unsigned xtag,
                            int xplain, int quad) {
  if (S <= 0 || Tn <= 0 || seq0 < 0 || !xbuf || xtag == 0 || (uint64_t)xtag + (uint64_t)Tn > 0xFFFFFFFFull)
    return hipErrorInvalidValue;
  LstmSync sy{};
  if (sync) {
    if (sync->nr < 1 || sync->nr > 16 || sync->seq_end[sync->nr - 1] < (sync->time_mode ? Tn : S))
      return hipErrorInvalidValue;
    for (int c = 1; c < sync->nr; ++c)
      if (sync->seq_end[c] <= sync->seq_end[c - 1]) return hipErrorInvalidValue;
    if (sync->gx_off < 0 || sync->gx_off >= Tn) return hipErrorInvalidValue;
    sy = *sync;
  }
  sy.xtag = xtag;
  sy.xplain = xplain;  // the handle's exchange-store policy (vap_create / vap_test_lstm_xplain)
  static const int hot = getenv("VAP_LSTM_HANDOFF") ? atoi(getenv("VAP_LSTM_HANDOFF")) : 0;  // diagnostics
  sy.handoff_trace = hot;
  static const int st0 = getenv("VAP_LSTM_STAMP_T0") ? atoi(getenv("VAP_LSTM_STAMP_T0")) : 100;
  sy.stamp_t0 = st0;
  const int groups = (S + NS - 1) / NS;
  static const bool stamps = getenv("VAP_LSTM_STAMPS") != nullptr;
  if (quad) {  // quads (b, b+8, b+16, b+24) of every 32 blocks; padding quads exit
    const dim3 gq(32 * ((groups + 7) / 8));
    // 96 KiB of (unused) dynamic LDS: one quarter per CU (its 4 waves hold half the register file, so two
    // quarters could otherwise share the SIMDs, and the persistent conv launches budget whole CUs for it)
    constexpr size_t excl = 96 * 1024;
    if (stamps)
      hipLaunchKernelGGL((lstm_quadb_kernel<true>), gq, dim3(256), excl, st, gx, seq0, S, Tn, (const chunk16*)whh_pair, out,
                         out_seq_stride, sy, (u32x4*)xbuf);
    else
      hipLaunchKernelGGL((lstm_quadb_kernel<false>), gq, dim3(256), excl, st, gx, seq0, S, Tn, (const chunk16*)whh_pair, out,
                         out_seq_stride, sy, (u32x4*)xbuf);
    return hipGetLastError();
  }
  const dim3 grid(16 * ((groups + 7) / 8));  // pairs (b, b + 8) of every 16 blocks; padding pairs exit
  if (stamps)
    hipLaunchKernelGGL((lstm_pair_kernel<true, true>), grid, dim3(512), 0, st, gx, seq0, S, Tn, (const chunk16*)whh_pair, out,
                       out_seq_stride, sy, (u32x4*)xbuf);
  else
    hipLaunchKernelGGL((lstm_pair_kernel<true, false>), grid, dim3(512), 0, st, gx, seq0, S, Tn, (const chunk16*)whh_pair, out,
                       out_seq_stride, sy, (u32x4*)xbuf);
  return hipGetLastError();
}
size_t lstm_quad_xbuf_bytes(int S) { return (size_t)((S + NS - 1) / NS) * Q_SLOT * 16; }

hipError_t launch_lstm_quad(const float* gx, int S, int Tn, const bf16* whh_quad, float* out, int64_t out_seq_stride,
                            hipStream_t st, void* xbuf, unsigned xtag, unsigned* err) {
  if (S <= 0 || Tn <= 0 || !xbuf || xtag == 0 || (uint64_t)xtag + (uint64_t)Tn >= 0xFFFFFFFFull) return hipErrorInvalidValue;
  // the per-lane buffer offsets of the output rows are 32-bit
  if ((int64_t)min(NS, S) * out_seq_stride * 4 >= 0x7FFFFFF0LL || (int64_t)Tn * HD > out_seq_stride) return hipErrorInvalidValue;
  const int groups = (S + NS - 1) / NS;
  const dim3 grid(32 * ((groups + 7) / 8));  // quads (b, b+8, b+16, b+24) of every 32 blocks; padding quads exit
  hipLaunchKernelGGL(lstm_quad_kernel, grid, dim3(256), 0, st, gx, S, Tn, (const chunk16*)whh_quad, out, out_seq_stride,
                     (u32x4*)xbuf, xtag, err);
  return hipGetLastError();
}
hipError_t launch_pack_whh_quad(const float* whh, bf16* packed, hipStream_t st) {
  hipLaunchKernelGGL(pack_whh_quad_kernel, dim3(256), dim3(256), 0, st, whh, packed);
  return hipGetLastError();
}
hipError_t launch_pack_whh_pair(const float* whh, bf16* packed, hipStream_t st) {
  hipLaunchKernelGGL(pack_whh_pair_kernel, dim3(256), dim3(256), 0, st, whh, packed, 1);
  return hipGetLastError();
}
hipError_t launch_pack_whh_resident(const float* whh, bf16* packed, hipStream_t st, bool prescaled) {
  hipLaunchKernelGGL(pack_whh_resident_kernel, dim3(256), dim3(256), 0, st, whh, packed, prescaled ? 1 : 0);
  return hipGetLastError();
}
hipError_t launch_pack_wih_prescaled(const float* wih, bf16* packed, const float* bih, const float* bhh, float* bias,
                                     hipStream_t st) {
  hipLaunchKernelGGL(pack_wih_prescaled_kernel, dim3(256), dim3(256), 0, st, wih, packed, bih, bhh, bias);
  return hipGetLastError();
}

template hipError_t launch_lstm<float>(const float*, int, int, const float*, float*, int64_t, hipStream_t);
template hipError_t launch_lstm<bf16>(const float*, int, int, const bf16*, bf16*, int64_t, hipStream_t);
template hipError_t launch_pack_whh<float>(const float*, float*, hipStream_t);
template hipError_t launch_pack_whh<bf16>(const float*, bf16*, hipStream_t);

hipError_t read_lstm_xcc(unsigned* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lstm_xcc), sizeof(g_lstm_xcc), 0, hipMemcpyDeviceToHost);
}
hipError_t read_lstm_handoff(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lstm_handoff), sizeof(g_lstm_handoff), 0, hipMemcpyDeviceToHost);
}
// diagnostics: copy the LSTM step stamps (8 workgroups x 4 steps x 5) to host memory
hipError_t read_lstm_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lstm_stamps), sizeof(g_lstm_stamps), 0, hipMemcpyDeviceToHost);
}
