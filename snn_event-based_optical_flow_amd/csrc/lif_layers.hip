// LIFFireNet cell kernels for gfx950: fused [LIF(l) on a halo tile] + conv3x3(l+1) + BN
// statistics forward, LIF(+pred) forward, and the matching backward kernels.
//
// Reference semantics (restated, see oracle/lif_ref.py):
//   cell   SNNtorch_ConvLIF(Recurrent).forward  models/SNNtorch_spiking_submodules.py:283-322, 515-567
//   neuron snntorch.Leaky (0.9.4), reset_delay=False, ATan surrogate (third-party, restated)
//   BN     torch BatchNorm2d train/eval (batch stats over B,H,W; running stats momentum update)
//   pred   models/submodules.py:ConvLayer (1x1 conv + bias, tanh)
//
// Layout: NHWC activations, state [2][B][H][W][C].  One 256-thread block owns an
// 8x32 pixel tile; halo rows are recomputed by neighbouring blocks (never stored).
#include <cmath>
#include <string>
#include <type_traits>

#include "snnflow_dev.h"
#include "snnflow_tile.h"

// Timing-attribution builds only (tools/kprobe.py): each set bit removes one stage,
// results are then meaningless.  0 in every shipped build.
#ifndef SNNFLOW_PROBE
#define SNNFLOW_PROBE 0
#endif
#define PROBE_OFF(bit) ((SNNFLOW_PROBE & (bit)) != 0)

// Phase-timestamp builds only (tools/ktrace.py, `make trace`): thread 0 of every block
// records the 100 MHz wall clock at phase boundaries of the C x C layer kernels.
// 0 in every shipped build.
#ifndef SNNFLOW_SP32
#define SNNFLOW_SP32 2  // threads per pixel of the C = 32 conv-layer kernels
#endif
#ifndef SNNFLOW_LATE_D_REC8
#define SNNFLOW_LATE_D_REC8 1  // C = 8 recurrent backward: LIF-backward inputs after the convs (no spill at 80 VGPRs)
#endif
#ifndef SNNFLOW_LATE_D_FF8
#define SNNFLOW_LATE_D_FF8 1  // C = 8 feed-forward LIF-fed backward: the same (A/B: 1.57-1.585 vs 1.593-1.595 ms)
#endif
#ifndef SNNFLOW_EARLY_G_REC8
#define SNNFLOW_EARLY_G_REC8 1  // C = 8 recurrent backward: BN-sum replicas ahead of the halo loads
#endif
#ifndef SNNFLOW_L32_WAVES
#define SNNFLOW_L32_WAVES 4  // min waves per SIMD of the C = 32 LIF-fed backward kernels
#endif
#ifndef SNNFLOW_TRACE
#define SNNFLOW_TRACE 0
#endif
#ifndef SNNFLOW_BWD_GATHER32
#define SNNFLOW_BWD_GATHER32 1  // C = 32 backward: batch-norm sums gathered by all threads, 2C for every block
#endif
#ifndef SNNFLOW_SWZ
#define SNNFLOW_SWZ 1  // C = 8 recurrent backward: bank-conflict-free LDS layouts of the packed x|s tile and dgrad staging
#endif
#ifndef SNNFLOW_TRACE_LAYER
// layer_bwd_body's stamps: off (with them k_bwd_slot<8> fails to compile on ROCm 7.2, "illegal VGPR to
// SGPR copy": the trace build stamps the forward slot kinds only)
#define SNNFLOW_TRACE_LAYER 0
#endif
#ifndef SNNFLOW_TRACE_MINGRID
#define SNNFLOW_TRACE_MINGRID 0  // stamp only launches of at least this many blocks (slot launches: 4 tasks)
#endif
#if SNNFLOW_TRACE
__device__ unsigned long long g_trace[4][4096][16];
#define TRACE_AT(on, kind, k)                                                                  \
    do {                                                                                      \
        if ((on) && threadIdx.x == 0 && blockIdx.x < 4096 && gridDim.x >= SNNFLOW_TRACE_MINGRID) \
            g_trace[kind][blockIdx.x][k] = wall_clock64();                                    \
    } while (0)
#else
#define TRACE_AT(on, kind, k) do { } while (0)
#endif

using namespace snnflow;

namespace {
thread_local std::string g_err;
}

int snnflow_set_error(int code, const char* msg) {
    g_err = msg;
    return code;
}

#define SNN_FAIL(code, msg) return snnflow_set_error((code), (msg))
#define SNN_CHECK_LAUNCH()                                                        \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) return snnflow_set_error((int)e_, hipGetErrorString(e_)); \
    } while (0)

namespace {

// dL/dm of the membrane input: v = beta*((1-r)*m) + I (zero reset) or beta*m + I - r*theta;
// r = H(m - theta) is detached (snntorch mem_reset).
__device__ inline float mem_grad(float gv, float m, const LifCoef& k, bool zero_reset) {
    const float gmp = gv * k.beta;
    if (!zero_reset) return gmp;
    const float r = (m - k.theta > 0.0f) ? 1.0f : 0.0f;
    return gmp * (1.0f - r);
}

// Per-channel neuron / BatchNorm parameters of one layer, loaded by threads c < C at
// kernel start, before the barrier-separated prologue: their round trip then overlaps
// the halo loads instead of following the batch-sum gather.
struct NeuronRegs { float w, b, beta, theta, rm, rv; };

template <bool SC1 = false>
__device__ inline NeuronRegs load_neuron(const snnflow_neuron& n, int C, bool lead) {
    NeuronRegs r = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int c = threadIdx.x;
    if (c < C) {
        r.w = n.bn_weight[c];
        r.b = n.bn_bias[c];
        r.beta = n.beta[c];
        r.theta = n.threshold[c];
        // running statistics: every block in eval mode, block 0 (the updater) in train mode
        // (SC1: the previous step's updater ran on another CU of this launch)
        if (n.running_mean && (!n.bn_train || lead)) {
            r.rm = ld1<SC1>(n.running_mean + c);
            r.rv = ld1<SC1>(n.running_var + c);
        }
    }
    return r;
}

// BatchNorm statistics of channel c from batch sums (train; sums[c] = S, sums[C+c] = SS)
// or running stats (eval): mean = S/N, var = SS/N - mean^2 (biased),
// invstd = 1/sqrt(var + eps) in fp64.
struct BnStat { float mean, invstd; double dmean, dvar; };

__device__ inline BnStat bn_stat(const snnflow_neuron& n, const NeuronRegs& r, const double* sums, int C, int c,
                                 double N) {
    BnStat st;
    if (n.bn_train) {
        st.dmean = sums[c] / N;
        st.dvar = sums[C + c] / N - st.dmean * st.dmean;
        if (st.dvar < 0.0) st.dvar = 0.0;
        st.mean = (float)st.dmean;
        st.invstd = (float)(1.0 / sqrt(st.dvar + n.eps));
    } else {
        st.dmean = r.rm;
        st.dvar = r.rv;
        st.mean = r.rm;
        st.invstd = (float)(1.0 / sqrt((double)r.rv + n.eps));
    }
    return st;
}

// Prologue of a LIF consumer: per-channel coefficients in LDS; block 0 also stores
// (mean, invstd) for the backward pass and performs the running-stat update
// (momentum, unbiased variance) and num_batches_tracked += 1 of torch's BatchNorm2d.
// `sums`: LDS totals from acc_gather (train mode only); r: load_neuron of this thread.
__device__ void lif_prologue(const snnflow_neuron& n, const NeuronRegs& r, const double* sums, int C, double N,
                             float* stats_out, LifCoef* coef, float* mean_out, bool lead, bool inlaunch = false) {
    const int c = threadIdx.x;
    if (c < C) {
        const BnStat st = bn_stat(n, r, sums, C, c, N);
        LifCoef k;
        k.alpha = st.invstd * r.w;
        k.shift = r.b - st.mean * k.alpha;
        k.beta = fminf(fmaxf(r.beta, 0.0f), 1.0f);
        k.theta = r.theta;
        coef[c] = k;
        if (mean_out) mean_out[c] = st.mean;
        if (lead) {
            if (stats_out) {
                stats_out[c] = st.mean;
                stats_out[C + c] = st.invstd;
            }
            if (n.bn_train && n.running_mean) {
                const double unb = N > 1.0 ? st.dvar * N / (N - 1.0) : st.dvar;
                n.running_mean[c] = (float)(n.momentum * st.dmean + (1.0 - n.momentum) * (double)r.rm);
                n.running_var[c] = (float)(n.momentum * unb + (1.0 - n.momentum) * (double)r.rv);
            }
        }
    }
    if (c == 0 && lead && n.bn_train && n.num_batches_tracked) {
        if (inlaunch)  // updated by several tasks of one persistent launch: coherent atomic
            __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(n.num_batches_tracked), 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        else
            n.num_batches_tracked[0] += 1;
    }
}

// Layer-l gradients of (gamma, bn bias, beta, threshold) [and pred] from the LIF-backward
// sums: gamma = dotp*invstd, bias = sum g, theta = -sum g, beta = sum g*m' (0 <= beta <= 1)
// (torch batch_norm_cpu_backward; snntorch Leaky; clamp backward passes on [0,1]).
// Block 0's inputs of neuron_grads other than the sums, loaded at kernel start (every
// load before any store: the destinations may alias as far as the compiler knows, and
// block 0's serial load->store chains would set the kernel's length).
struct NeuronGradRegs { float inv, be, o0, o1, o2, o3, op; };

__device__ inline NeuronGradRegs load_neuron_grad(const snnflow_neuron& n, const float* stats, int C,
                                                  const snnflow_neuron_grad& ng, int accumulate, int has_pred,
                                                  float* g_pred_w, float* g_pred_b, bool lead) {
    NeuronGradRegs r = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (!lead) return r;
    const int c = threadIdx.x;
    if (c < C) {
        r.inv = stats[C + c];
        r.be = n.beta[c];
        if (accumulate) {
            r.o0 = ng.bn_weight[c]; r.o1 = ng.bn_bias[c]; r.o2 = ng.threshold[c]; r.o3 = ng.beta[c];
        }
    }
    if (has_pred && accumulate && c < 2 * C + 2) r.op = (c < 2 * C) ? g_pred_w[c] : g_pred_b[c - 2 * C];
    return r;
}

__device__ void neuron_grads(const NeuronGradRegs& r, const double* sums, int C, const snnflow_neuron_grad& ng,
                             int has_pred, float* g_pred_w, float* g_pred_b, bool lead) {
    if (!lead) return;
    const int c = threadIdx.x;
    if (c < C) {
        const double gsum = sums[c], dotp = sums[C + c], gbm = sums[2 * C + c];
        const float gw = (float)(dotp * (double)r.inv);
        const float gb = (float)gsum;
        // (no prediction: sums[3C + c] holds the membrane-output part of a detach=False cell, else 0)
        const float gth = has_pred ? -(float)gsum : (float)(sums[3 * C + c] - gsum);
        const float gbe = (r.be >= 0.0f && r.be <= 1.0f) ? (float)gbm : 0.0f;
        ng.bn_weight[c] = r.o0 + gw;
        ng.bn_bias[c] = r.o1 + gb;
        ng.threshold[c] = r.o2 + gth;
        ng.beta[c] = r.o3 + gbe;
    }
    if (has_pred && c < 2 * C + 2) {
        float* dst = (c < 2 * C) ? g_pred_w + c : g_pred_b + (c - 2 * C);
        *dst = r.op + (float)sums[3 * C + c];
    }
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
// Up to 16 descriptors passed by value in the kernarg segment; blockIdx.y picks one
// through constant-index selects (a dynamic index would copy the array to scratch).
template <typename D>
struct DescBatch {
    D d[SNNFLOW_MAX_BATCH];
    __device__ inline D pick(int k) const {
        D r = d[0];
#pragma unroll
        for (int i = 1; i < SNNFLOW_MAX_BATCH; ++i)
            if (k == i) r = d[i];
        return r;
    }
};

// Matrix-core operand geometry of a KIN x NOUT 3x3 conv at run time (Bf3Geo / bf3_k).
struct FragGeo {
    int gpt, tpi, ipt, ni, nnt;
    __host__ __device__ FragGeo(int kin, int nout) {
        gpt = kin / 8;
        tpi = gpt >= 4 ? 1 : 4 / gpt;
        ipt = gpt >= 4 ? gpt / 4 : 1;
        ni = ((9 + tpi - 1) / tpi) * ipt;
        nnt = (nout + 15) / 16;
    }
    __host__ __device__ int halfs() const { return ni * nnt * 3 * 512; }
    __device__ void k(int i, int g, int& tap, int& c0) const {
        if (gpt >= 4) {
            tap = i / ipt;
            c0 = ((i % ipt) * 4 + g) * 8;
        } else {
            tap = i * tpi + g / gpt;
            c0 = (g % gpt) * 8;
        }
    }
};

// Fragment element e (chunk, n-tile, lane, j) of a KIN x NOUT conv: the three bf16 parts of
// W(tap, n, k = c0 + j) at frag[((chunk * nnt + nt) * 3 + part) * 512 + lane * 8 + j]
// (FragStage's layout, in global memory).  fwd: n = co, k = ci; !fwd (input gradient): n = ci, k = co.
__device__ inline void prep_frag(const snnflow_prep_desc& d, int e, bool fwd) {
    const int c = d.c, cin = d.cin;
    const FragGeo G(fwd ? cin : c, fwd ? c : cin);
    if (e >= G.ni * G.nnt * 512) return;
    const int j = e & 7, lane = (e >> 3) & 63, rest = e >> 9;
    const int nt = rest % G.nnt, ch = rest / G.nnt, n = nt * 16 + (lane & 15);
    int tap, c0;
    G.k(ch, lane >> 4, tap, c0);
    const int kk = c0 + j, nout = fwd ? c : cin;
    float w = 0.0f;
    if (tap < 9 && n < nout) w = fwd ? d.w[(n * cin + kk) * 9 + tap] : d.w[(kk * cin + n) * 9 + tap];
    const __bf16 h = (__bf16)w;
    const float r1 = w - (float)h;
    const __bf16 md = (__bf16)r1;
    const __bf16 lo = (__bf16)(r1 - (float)md);
    uint16_t* f = (fwd ? d.frag_fwd : d.frag_bwd) + (rest * 3) * 512 + (e & 511);
    f[0] = __builtin_bit_cast(uint16_t, h);
    f[512] = __builtin_bit_cast(uint16_t, md);
    f[1024] = __builtin_bit_cast(uint16_t, lo);
}

__global__ void k_prep_weights(DescBatch<snnflow_prep_desc> batch) {
    const snnflow_prep_desc d = batch.pick(blockIdx.y);
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int c = d.c, cin = d.cin, n = c * cin * 9;
    if (d.w && e < n) {
        const int k = e % 9, ci = (e / 9) % cin, co = e / (9 * cin);
        const float v = d.w[e];
        d.wt_fwd[(k * cin + ci) * c + co] = v;
        d.wt_bwd[(k * c + co) * cin + ci] = v;
    }
    if (d.w && d.frag_fwd) prep_frag(d, e, true);
    if (d.w && d.frag_bwd) prep_frag(d, e, false);
    if (d.threshold && e < d.thr_n) {
        const float t = d.threshold[e];
        d.threshold[e] = (t < 0.01f) ? 0.01f : t;
    }
    if (d.zero) {
        for (int64_t i = e; i < d.zero_n; i += (int64_t)gridDim.x * blockDim.x) d.zero[i] = 0.0;
    }
}

// The C x C conv layers (C = 8, 16, 32) run their convolutions on the matrix cores.
template <int CIN, int C>
constexpr bool kMfma = CIN == C && C % 8 == 0;
// ... with their weights staged in LDS up to C = 16 (C = 32: 36 KB per conv, read from L2)
template <int CIN, int C>
constexpr bool kWlds = kMfma<CIN, C> && C <= 16;

// LIF of one float4 of channels [4q, 4q+4) (coefficients from LDS).
struct Lif4 { float4 s, mout; };

__device__ inline Lif4 lif_step4(const float4& y, const float4& m, const LifCoef* coef, bool zr) {
    const LifOut o0 = lif_step(y.x, m.x, coef[0], zr);
    const LifOut o1 = lif_step(y.y, m.y, coef[1], zr);
    const LifOut o2 = lif_step(y.z, m.z, coef[2], zr);
    const LifOut o3 = lif_step(y.w, m.w, coef[3], zr);
    Lif4 r;
    r.s = make_float4(o0.s, o1.s, o2.s, o3.s);
    r.mout = make_float4(o0.mout, o1.mout, o2.mout, o3.mout);
    return r;
}

template <bool F, int C, int NTB>
struct FragFloats { static constexpr int v = 0; };
template <int C, int NTB>
struct FragFloats<true, C, NTB> { static constexpr int v = (FragStage<C, C, NTB>::HALFS / 2 + 3) / 4 * 4; };

// LDS of one conv_fwd block (floats, 16-B aligned parts): halo tile, [s_prev halo tile],
// [weights of the ff / rec convs].  Carved out of one pool so that a wavefront launch can
// run several variants over the same allocation.
template <int CIN, int C, bool LIF_IN, bool REC, int SPLIT>
struct ConvFwdLds {
    static constexpr int NTB = NT * SPLIT, PI_ = Pad<CIN>::v, PC = Pad<C>::v;
    static constexpr bool PF_REC = REC && Prefetch<C, NTB>::on;  // s_prev halo in registers + own LDS tile
    static constexpr int PMAX = (REC && !PF_REC && PC > PI_) ? PC : PI_;
    // C = 8 spike convs: B operand pre-split into bf16 fragments once per block (FragStage);
    // otherwise f32 weights in LDS up to C = 16 (kWlds)
    static constexpr bool BT = LIF_IN && kMfma<CIN, C>;  // LIF spikes of the halo as a bf16 tile
    static constexpr bool FRAG = BT && C == 8;
    static constexpr bool WL = kWlds<CIN, C> && !FRAG;
    static constexpr int FRAGF = FragFloats<FRAG, C, NTB>::v;
    // BT: the halo spikes as a bf16 tile [HN][C] (exact 0/1, a lane's MFMA A operand in one 16-B
    // read); the output staging after the convs (mfma_store, f32 [NT][PC]) reuses the pool
    static constexpr int TILE = BT ? (HN * C / 2 + 3) / 4 * 4 : (HN * PMAX + 3) / 4 * 4;
    static constexpr int RTILE = PF_REC ? HN * PC : 0;
    static constexpr int WFF = WL ? 9 * C * C : FRAGF, WREC = REC ? (WL ? 9 * C * C : FRAGF) : 0;
    static constexpr int BODY = TILE + RTILE + WFF + WREC;
    static constexpr int FLOATS = (BT && BODY < NT * PC) ? NT * PC : BODY;
    static_assert(!BT || !REC || PF_REC, "bf16 spike tile: s_prev needs its own tile");
};

template <int CIN, int C, bool LIF_IN, bool REC, int SPLIT, bool SC1 = false>
__device__ void conv_fwd_body(const snnflow_conv_fwd_args& a, const Grid g, float* lds) {
    using L = ConvFwdLds<CIN, C, LIF_IN, REC, SPLIT>;
    constexpr int NTB = NT * SPLIT, CO = C / SPLIT;
    static_assert(CO % 4 == 0, "output channels per group: multiple of 4");
    constexpr int PI_ = L::PI_, PC = L::PC;
    constexpr bool PF_REC = L::PF_REC;
    float* tile = lds;
    [[maybe_unused]] float* rtile = lds + L::TILE;
    [[maybe_unused]] float* wl_ff = rtile + L::RTILE;
    [[maybe_unused]] float* wl_rec = wl_ff + L::WFF;
    __shared__ LifCoef coef[LIF_IN ? CIN : 1];

    const int tid = threadIdx.x, pt = tid % NT, ty = pt / TW, tx = pt - ty * TW;
    const int part = thread_part(), co0 = part * CO;
    const int H = a.H, W = a.W;
    const Tile tl = block_tile(H, W, g);
    // previous-step spikes: an fp32 NHWC plane (s_prev) or a spike bit plane (s_prev_bits, ABI 39)
    [[maybe_unused]] constexpr bool SBITS = REC && (C == 8 || C == 16 || C == 32);
    const bool rec_bits = SBITS && a.s_prev_bits != nullptr;
    const bool has_rec = REC && (a.s_prev != nullptr || rec_bits);
    [[maybe_unused]] constexpr bool TR = LIF_IN && CIN == C;
    [[maybe_unused]] constexpr int TK = REC ? 1 : 0;
    TRACE_AT(TR, TK, 0);
    __shared__ int rec_bad[1];
    if (tid == 0) rec_bad[0] = 0;  // (read after the barrier that follows the exactness test)

    // 1. issue every global load of the tile before any use: the BN-sum replicas first (their
    //    reduction and the coefficients then overlap the halo loads), weights for LDS next
    AccGather<LIF_IN ? 2 * CIN : 1> gat;
    NeuronRegs nr = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (LIF_IN) {
        if (a.prev.bn_train) acc_gather_load<2 * CIN, SC1>(a.prev_acc, 2 * CIN, gat);
        nr = load_neuron<SC1>(a.prev, CIN, g.bid == 0);
    }
    constexpr bool WL = L::WL, FRAG = L::FRAG;
    WStage<WL ? 9 * C * C : 1, NTB> sw_ff, sw_rec;
    FragStage<FRAG ? C : 8, FRAG ? C : 8, FRAG ? NTB : 64> fs_ff, fs_rec;
    if constexpr (WL) {
        sw_ff.load(a.wt_ff_t);
        if constexpr (REC) {
            if (has_rec) sw_rec.load(a.wt_rec_t);
        }
    }
    if constexpr (FRAG) {
        fs_ff.load(a.wt_ff_t);
        if constexpr (REC) {
            if (has_rec) fs_rec.load(a.wt_rec_t);
        }
    }
    float4 rs[PF_REC ? Halo4<C, NTB>::R : 1];
    [[maybe_unused]] unsigned rsb[PF_REC && SBITS ? Halo4<C, NTB>::R : 1];
    if constexpr (PF_REC) {
        if constexpr (SBITS) {
            if (rec_bits) halo_load_bits<C, NTB>(a.s_prev_bits, tl, H, W, rsb);
            else if (has_rec) halo_load<C, NTB, (C <= 8), SC1>(a.s_prev, tl, H, W, rs);
        } else {
            if (has_rec) halo_load<C, NTB, (C <= 8), SC1>(a.s_prev, tl, H, W, rs);
        }
    }
    if constexpr (LIF_IN) {
        constexpr int R = Halo4<CIN, NTB>::R, Q = CIN / 4;
        float4 ry[R], rm[R];
        halo_load<CIN, NTB, (CIN <= 8), SC1>(a.prev_y, tl, H, W, ry);
        if (a.prev_mem) halo_load<CIN, NTB, (CIN <= 8), SC1>(a.prev_mem, tl, H, W, rm);
        else zero4(rm, R);
        __shared__ double sums[2 * CIN];
        if (a.prev.bn_train) acc_gather_reduce<2 * CIN>(gat, sums);
        lif_prologue(a.prev, nr, sums, CIN, (double)a.B * H * W, a.prev_stats, coef, nullptr, g.bid == 0, SC1);
        __syncthreads();
        // (stores issued after the gather: CDNA's vmcnt counts stores, so zeroing before the
        // gather made its wait include the store acknowledgements)
        zero_consumed(a.zero0, a.zero1, a.zero_n, g);
        TRACE_AT(TR, TK, 1);
        // 2. LIF of the previous layer over the halo; interior pixels also write its state.
        //    Element e = tid + i*NTB has channel quad e % Q = tid % Q (NTB % Q == 0): the four
        //    coefficients come out of LDS once, and the reset flavour is a loop version.
        static_assert(NTB % Q == 0, "constant channel quad per thread");
        const int64_t plane4 = (int64_t)a.B * H * W * Q;
        float4* st4 = reinterpret_cast<float4*>(a.prev_state);
        const int qt = tid % Q;
        const LifCoef kc[4] = {coef[4 * qt], coef[4 * qt + 1], coef[4 * qt + 2], coef[4 * qt + 3]};
        // the previous layer's spike bit plane (ABI 39): interior pixels, one word per pixel
        constexpr bool OBITS = CIN == C && (C == 8 || C == 16 || C == 32);
        uint8_t* const obits = OBITS ? a.prev_spk_bits : nullptr;
        auto halo_lif = [&](auto zr_c) {
            constexpr bool ZR = decltype(zr_c)::value;
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const int e = tid + i * NTB;
                if (e < Halo4<CIN, NTB>::E) {
                    const int p = e / Q;
                    const int r = p / HWD, cc = p - r * HWD;
                    const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
                    const bool img = in_image(h, w, H, W), inner = img && r >= 1 && r <= TH && cc >= 1 && cc <= TW;
                    float4 sv = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (img) {
                        const Lif4 o = lif_step4(ry[i], rm[i], kc, ZR);
                        sv = o.s;
                        if (inner) {
                            const int64_t k = (((int64_t)tl.b * H + h) * W + w) * Q + qt;
                            // write-through: read again only at the next time step (measured -1 us per launch)
                            st_state4(st4, k, o.mout);
                            if (!a.state_spk_skip) st_state4(st4, plane4 + k, o.s);
                        }
                    }
                    if constexpr (OBITS) {
                        if (obits != nullptr) {
                            const unsigned wb = spk_pack_wave<CIN>(sv, tid & 63);
                            if (inner && qt == 0) spk_store_bits<CIN>(obits, ((int64_t)tl.b * H + h) * W + w, wb);
                        }
                    }
                    if constexpr (L::BT) {
                        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                        const bf16x4 sb = {(__bf16)sv.x, (__bf16)sv.y, (__bf16)sv.z, (__bf16)sv.w};
                        *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(tile) + p * CIN + 4 * qt) = sb;
                    } else {
                        *reinterpret_cast<float4*>(tile + p * PI_ + 4 * qt) = sv;
                    }
                }
            }
        };
        if (a.prev.zero_reset) halo_lif(std::true_type{});
        else halo_lif(std::false_type{});
    } else {
        stage_strided<CIN, NTB>(a.x, a.xs_b, a.xs_c, a.xs_h, a.xs_w, tl, H, W, tile);
        zero_consumed(a.zero0, a.zero1, a.zero_n, g);
    }
    if constexpr (WL) {
        sw_ff.store(wl_ff);
        if constexpr (REC) {
            if (has_rec) sw_rec.store(wl_rec);
        }
    }
    if constexpr (FRAG) {
        fs_ff.store(reinterpret_cast<__bf16*>(wl_ff));
        if constexpr (REC) {
            if (has_rec) fs_rec.store(reinterpret_cast<__bf16*>(wl_rec));
        }
    }
    // previous-step spikes exact in bf16 (0/1; always so on the engine path) -> bf16 MFMA; a wave with an
    // inexact value sets an LDS flag (cleared at kernel start) instead of __syncthreads_and's barriers
    if constexpr (PF_REC && SBITS) {
        if (rec_bits) {  // exact 0/1 by construction
            constexpr int Q = C / 4;
#pragma unroll
            for (int i = 0; i < Halo4<C, NTB>::R; ++i) {
                const int e = tid + i * NTB;
                if (e < Halo4<C, NTB>::E) {
                    const int p = e / Q, q = e - p * Q;
                    *reinterpret_cast<float4*>(rtile + p * Pad<C>::v + 4 * q) = spk_quad<C>(rsb[i], q);
                }
            }
        }
    }
    if constexpr (PF_REC) {
        if (has_rec && !(SBITS && rec_bits)) {
            halo_store<C, NTB>(rtile, rs);
            bool ok = true;
#pragma unroll
            for (int i = 0; i < Halo4<C, NTB>::R; ++i)
                ok = ok && exact_bf16(rs[i].x) && exact_bf16(rs[i].y) && exact_bf16(rs[i].z) && exact_bf16(rs[i].w);
            if (__builtin_amdgcn_ballot_w64(!ok) != 0 && (tid & 63) == 0) rec_bad[0] = 1;
        }
    }
    __syncthreads();
    const bool rec_bf = PF_REC && has_rec && rec_bad[0] == 0;
    TRACE_AT(TR, TK, 2);

    float y[CO];
    if constexpr (kMfma<CIN, C>) {
        // matrix-core implicit GEMM over the whole tile (weights in the [tap][c][cin] layout);
        // the sums come back through LDS, aliasing `tile`, in this thread's pixel/channel order
        constexpr int NW = NTB / 64;
        constexpr int NG = C >= 32 ? 2 : 1;  // C = 32: waves split the output channels too
        MfmaAcc<C, C, NW, NG> af, ar;
        af.zero();
        if (!PROBE_OFF(16)) {
            const float* wf = WL ? wl_ff : a.wt_ff_t;
            if constexpr (FRAG)
                mfma_conv3x3_bf3f<C, C, NW>(reinterpret_cast<const __bf16*>(tile), reinterpret_cast<const __bf16*>(wl_ff), af);
            else if constexpr (L::BT) {  // spikes of layer l-1
                const __bf16* tb = reinterpret_cast<const __bf16*>(tile);
                if (a.wf_ff) mfma_conv3x3_bf3g<C, C, NW, __bf16, NG>(tb, reinterpret_cast<const __bf16*>(a.wf_ff), af);
                else mfma_conv3x3_bf3<C, C, NW, __bf16, NG>(tb, wf, af);
            }
            else mfma_conv3x3<C, C, false, NW, NG>(tile, wf, af);
        }
        bool rec_on = false;
        if constexpr (REC) {
            if (has_rec) {
                rec_on = true;
                const float* rt = tile;
                if constexpr (PF_REC) {
                    rt = rtile;
                } else {
                    __syncthreads();
                    if constexpr (SBITS) {
                        if (rec_bits) stage_nhwc_bits<C, NTB>(a.s_prev_bits, tl, H, W, tile);
                        else stage_nhwc<C, NTB>(a.s_prev, tl, H, W, tile);
                    } else {
                        stage_nhwc<C, NTB>(a.s_prev, tl, H, W, tile);
                    }
                    __syncthreads();
                }
                ar.zero();
                if (!PROBE_OFF(16)) {
                    const float* wr = WL ? wl_rec : a.wt_rec_t;
                    if constexpr (FRAG) {
                        if (rec_bf) mfma_conv3x3_bf3f<C, C, NW>(rt, reinterpret_cast<const __bf16*>(wl_rec), ar);
                        else mfma_conv3x3<C, C, false, NW>(rt, a.wt_rec_t, ar);  // non-binary s_prev
                    } else {
                        if (rec_bf && a.wf_rec)
                            mfma_conv3x3_bf3g<C, C, NW, float, NG>(rt, reinterpret_cast<const __bf16*>(a.wf_rec), ar);
                        else if (rec_bf) mfma_conv3x3_bf3<C, C, NW, float, NG>(rt, wr, ar);
                        else mfma_conv3x3<C, C, false, NW, NG>(rt, wr, ar);
                    }
                }
            }
        }
        __syncthreads();
        if (rec_on) mfma_store<true>(af, ar, tile);  // ff + rec (:540)
        else mfma_store<false>(af, ar, tile);
        __syncthreads();
        const float* yl = tile + pt * PC + co0;
#pragma unroll
        for (int co = 0; co < CO; co += 4) {
            const float4 v = *reinterpret_cast<const float4*>(yl + co);
            y[co] = v.x; y[co + 1] = v.y; y[co + 2] = v.z; y[co + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int co = 0; co < CO; ++co) y[co] = 0.0f;
        if (!PROBE_OFF(16)) conv_acc<CIN, C, CO>(tile, a.wt_ff, ty, tx, co0, y);

        if constexpr (REC) {
            if (has_rec) {
                const float* rt = tile;
                if constexpr (PF_REC) {
                    rt = rtile;
                } else {
                    __syncthreads();
                    if constexpr (SBITS) {
                        if (rec_bits) stage_nhwc_bits<C, NTB>(a.s_prev_bits, tl, H, W, tile);
                        else stage_nhwc<C, NTB>(a.s_prev, tl, H, W, tile);
                    } else {
                        stage_nhwc<C, NTB>(a.s_prev, tl, H, W, tile);
                    }
                    __syncthreads();
                }
                float r[CO];
#pragma unroll
                for (int co = 0; co < CO; ++co) r[co] = 0.0f;
                if (!PROBE_OFF(16)) conv_acc<C, C, CO>(rt, a.wt_rec, ty, tx, co0, r);
#pragma unroll
                for (int co = 0; co < CO; ++co) y[co] = y[co] + r[co];  // ff + rec (:540)
            }
        }
    }

    TRACE_AT(TR, TK, 3);
    const int h = tl.h0 + ty, w = tl.w0 + tx;
    const bool in = (h < H) && (w < W);
    if (in) {
        float* yp = a.y + (((int64_t)tl.b * H + h) * W + w) * C + co0;
#pragma unroll
        for (int co = 0; co < CO; co += 4)
            *reinterpret_cast<float4*>(yp + co) = make_float4(y[co], y[co + 1], y[co + 2], y[co + 3]);
    }
    if (a.acc) {
        float v[2 * CO];
#pragma unroll
        for (int co = 0; co < CO; ++co) {
            const float yy = in ? y[co] : 0.0f;
            v[co] = yy;
            v[CO + co] = yy * yy;
        }
        double* acc = acc_shard(a.acc, 2 * C, g.bid);
        if (!PROBE_OFF(4))
            block_atomic_sum_parts<2 * CO, SPLIT>(v, [acc](int pp, int j) {
                return acc + (j < CO ? pp * CO + j : C + pp * CO + (j - CO));
            });
    }
    TRACE_AT(TR, TK, 4);
}

template <int CIN, int C, bool LIF_IN, bool REC, int SPLIT>
__global__ __launch_bounds__(NT * SPLIT) void k_conv_fwd(snnflow_conv_fwd_args a) {
    __shared__ __attribute__((aligned(16))) float pool[ConvFwdLds<CIN, C, LIF_IN, REC, SPLIT>::FLOATS];
    conv_fwd_body<CIN, C, LIF_IN, REC, SPLIT>(a, hw_grid(), pool);
}

// LIF (+ 1x1 pred conv + tanh) over pixels: one thread per pixel, all C channels.
// NTH threads (= pixels) per block: NT for its own launch, NT * 2 inside a wavefront launch.
template <int C, bool PRED, int NTH, bool SC1 = false>
__device__ void lif_fwd_body(const snnflow_lif_fwd_args& a, const Grid g) {
    constexpr int Q = C / 4;
    __shared__ LifCoef coef[C];
    const int tid = threadIdx.x;
    const int64_t HWp = (int64_t)a.H * a.W, npix = (int64_t)a.B * HWp, plane4 = npix * Q;
    const int64_t p = (int64_t)g.bid * NTH + tid;
    const bool act = p < npix;
    const float4* y4 = reinterpret_cast<const float4*>(a.y);
    const float4* m4 = reinterpret_cast<const float4*>(a.mem);
    const int64_t pc = act ? p : npix - 1;  // unconditional 16-B loads
    // BN-sum replicas and per-channel parameters first: their math then overlaps the pixel loads
    AccGather<2 * C> gat;
    if (a.n.bn_train) acc_gather_load<2 * C, SC1>(a.acc, 2 * C, gat);
    const NeuronRegs nr = load_neuron<SC1>(a.n, C, g.bid == 0);
    float4 yv[Q], mv[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        yv[q] = ld4<SC1>(y4, pc * Q + q);
        mv[q] = ld4_or_zero_sc<SC1>(m4, y4, pc * Q + q);
    }
    __shared__ double sums[2 * C];
    if (a.n.bn_train) acc_gather_reduce<2 * C>(gat, sums);
    lif_prologue(a.n, nr, sums, C, (double)npix, a.stats, coef, nullptr, g.bid == 0, SC1);
    __syncthreads();
    zero_consumed(a.zero0, a.zero1, a.zero_n, g);  // after the gather (vmcnt counts stores)
    if (!act) return;
    const bool zr = a.n.zero_reset != 0;
    float4* st4 = reinterpret_cast<float4*>(a.state);
    float s[C];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const Lif4 o = lif_step4(yv[q], mv[q], coef + 4 * q, zr);
        st4[p * Q + q] = o.mout;  // plain: write-through measured slower in this streaming kernel
        if (!a.state_spk_skip) st4[plane4 + p * Q + q] = o.s;
        s[4 * q] = o.s.x; s[4 * q + 1] = o.s.y; s[4 * q + 2] = o.s.z; s[4 * q + 3] = o.s.w;
    }
    if constexpr (PRED) {
        const int64_t b = p / HWp, hw = p - b * HWp;
        const cfloat_ptr pw = as_const(a.pred_w);
#pragma unroll
        for (int o = 0; o < 2; ++o) {
            float acc = 0.0f;
#pragma unroll
            for (int c = 0; c < C; ++c) acc = fmaf(pw[o * C + c], s[c], acc);
            a.flow[(b * 2 + o) * HWp + hw] = tanhf(acc + a.pred_b[o]);
        }
    }
}

template <int C, bool PRED>
__global__ __launch_bounds__(NT) void k_lif_fwd(snnflow_lif_fwd_args a) {
    lif_fwd_body<C, PRED, NT>(a, hw_grid());
}

// Surrogate-gradient backward of the top LIF (+ pred): one thread per pixel; BN/neuron
// sums into acc (block partials, fp64 atomics).
// dL/dv of snn.Leaky when the membrane output also carries gradient g_mo (detach=False,
// SNNtorch_spiking_submodules.py:309-311), from g_s (spike output) and the reset r = H(m - theta)
// (detached): zero reset m_out = v (1 - s + r) -> g_v = sg (g_s - v g_mo) + g_mo (1 - s + r);
// subtract reset m_out = v - (s - r) theta -> g_v = sg (g_s - theta g_mo) + g_mo.  The threshold
// then receives -sum g_v (+ -sum r g_v, subtract: snnflow_lif_theta_subtract) plus gth =
// g_mo (1 - s + r), summed separately.
struct MemOutGrad { float gv, gth; };

__device__ inline MemOutGrad mem_out_grad(float gs, float gmo, float m, const LifOut& o, const LifCoef& k, bool zr) {
    const float sg = atan_sg(o.v - k.theta);
    const float r = (m - k.theta > 0.0f) ? 1.0f : 0.0f;
    const float keep = (1.0f - o.s) + r;
    MemOutGrad d;
    d.gv = zr ? sg * (gs - o.v * gmo) + gmo * keep : sg * (gs - k.theta * gmo) + gmo;
    d.gth = gmo * keep;
    return d;
}

template <int C, bool PRED, int NTH>
__device__ void lif_bwd_body(const snnflow_lif_bwd_args& a, const Grid g) {
    // sums: (g, (y - mean) g, g m') per channel, then [pred: (gpre0 s, gpre1 s) per channel, gpre0,
    // gpre1] or [no pred: the membrane-gradient threshold part g_mo (1 - s + r) per channel]
    constexpr int NV = 3 * C + (PRED ? 2 * C + 2 : C), Q = C / 4;
    static_assert(NTH % NT == 0, "whole 256-thread parts");
    __shared__ LifCoef coef[C];
    __shared__ float meanv[C];
    const int tid = threadIdx.x;
    const int64_t HWp = (int64_t)a.H * a.W, npix = (int64_t)a.B * HWp, plane4 = npix * Q;
    const int64_t p = (int64_t)g.bid * NTH + tid;
    const bool act = p < npix;
    const int64_t pc = act ? p : npix - 1;
    const int64_t b = pc / HWp, hw = pc - b * HWp;
    // per-channel coefficients first (their loads then do not wait behind the pixel loads)
    LifCoef kc = {0.f, 0.f, 0.f, 0.f};
    float mu = 0.f;
    if (tid < C) {
        kc = lif_coef(a.n, a.stats, C, tid);
        mu = a.stats[tid];
    }
    float4 yv[Q], mv[Q], gs[Q];
    [[maybe_unused]] float4 gmo4[PRED ? 1 : Q];
    const float4* y4 = reinterpret_cast<const float4*>(a.y);
    const float4* m4 = reinterpret_cast<const float4*>(a.mem);
    const float4* go4 = reinterpret_cast<const float4*>(a.g_out);
    const float4* gst4 = reinterpret_cast<const float4*>(a.g_state);
    [[maybe_unused]] const bool mgi = !PRED && a.mem_grad_in && gst4;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        yv[q] = y4[pc * Q + q];  // unconditional 16-B loads (clamped pixel)
        mv[q] = ld4_or_zero(m4, y4, pc * Q + q);
        float4 g = ld4_or_zero(go4, y4, pc * Q + q);
        const float4 t = ld4_or_zero(gst4 ? gst4 + plane4 : nullptr, y4, pc * Q + q);
        if (gst4) g = make_float4(g.x + t.x, g.y + t.y, g.z + t.z, g.w + t.w);
        gs[q] = g;
        if constexpr (!PRED) gmo4[q] = ld4_or_zero(mgi ? gst4 : nullptr, y4, pc * Q + q);
    }
    float fl[2] = {0.f, 0.f}, gf[2] = {0.f, 0.f};
    if constexpr (PRED) {
        if (a.g_flow) {
#pragma unroll
            for (int o = 0; o < 2; ++o) {
                fl[o] = a.flow[(b * 2 + o) * HWp + hw];
                gf[o] = a.g_flow[b * a.gflow_sb + o * a.gflow_sc + hw];
            }
        }
    }
    if (tid < C) {
        coef[tid] = kc;
        meanv[tid] = mu;
    }
    __syncthreads();
    const bool zr = a.n.zero_reset != 0;
    float v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = 0.0f;
    float gpre[2] = {0.0f, 0.0f};
    if constexpr (PRED) {
        if (act && a.g_flow) {
#pragma unroll
            for (int o = 0; o < 2; ++o) gpre[o] = gf[o] * (1.0f - fl[o] * fl[o]);  // tanh backward
        }
    }
    if (act) {
        const cfloat_ptr pw = as_const(a.pred_w);
        float4* gc4 = reinterpret_cast<float4*>(a.g_cur);
        float4* gm4 = reinterpret_cast<float4*>(a.g_mem);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const float yi[4] = {yv[q].x, yv[q].y, yv[q].z, yv[q].w};
            const float mi[4] = {mv[q].x, mv[q].y, mv[q].z, mv[q].w};
            const float gi[4] = {gs[q].x, gs[q].y, gs[q].z, gs[q].w};
            float go[4], gmo[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = 4 * q + j;
                float g = gi[j];
                if constexpr (PRED) {
                    if (a.g_flow) g = g + (pw[c] * gpre[0] + pw[C + c] * gpre[1]);
                }
                const LifOut o = lif_step(yi[j], mi[j], coef[c], zr);
                float gv = atan_sg(o.v - coef[c].theta) * g;
                if constexpr (!PRED) {
                    if (mgi) {
                        const float gm = j == 0 ? gmo4[q].x : (j == 1 ? gmo4[q].y : (j == 2 ? gmo4[q].z : gmo4[q].w));
                        const MemOutGrad d = mem_out_grad(g, gm, mi[j], o, coef[c], zr);
                        gv = d.gv;
                        v[3 * C + c] += d.gth;
                    }
                }
                go[j] = gv;
                gmo[j] = mem_grad(gv, mi[j], coef[c], zr);
                v[c] += gv;
                v[C + c] += (yi[j] - meanv[c]) * gv;
                v[2 * C + c] += gv * o.mprime;
                if constexpr (PRED) {
                    v[3 * C + c] += gpre[0] * o.s;
                    v[4 * C + c] += gpre[1] * o.s;
                }
            }
            gc4[p * Q + q] = make_float4(go[0], go[1], go[2], go[3]);
            if (gm4) gm4[p * Q + q] = make_float4(gmo[0], gmo[1], gmo[2], gmo[3]);
        }
        if constexpr (PRED) {
            v[5 * C] += gpre[0];
            v[5 * C + 1] += gpre[1];
        }
    }
    double* acc = acc_shard(a.acc, SNNFLOW_BWD_ACC(C), g.bid);
    if (!PROBE_OFF(4)) block_atomic_sum_parts<NV, NTH / NT>(v, [acc](int, int j) { return acc + j; });
    zero_consumed(a.zero0, a.zero1, a.zero_n, g);  // last: no load waits behind these stores
}

template <int C, bool PRED>
__global__ __launch_bounds__(NT) void k_lif_bwd(snnflow_lif_bwd_args a) {
    lif_bwd_body<C, PRED, NT>(a, hw_grid());
}

// Standalone (per-step) LIF launches: one thread per (pixel, channel quad), `items` pixels of
// the block's contiguous range per thread.  The one-thread-per-pixel bodies above keep a pixel's
// C channels in one thread (the wavefront launches' C = 8 top task); at C = 16 / 32 that
// serialises 2-4x the loads and stores per thread and, backward, reduces 3C + 2C + 2 sums per
// thread through the block.  Here a thread holds one float4 of each tensor and 12 (+ 10 with
// the prediction) running sums; lanes of equal quad are reduced once per block.
// Grids of one resident round (no tail): forward 6 blocks per CU (58-72 VGPRs), backward 4
// (78-108 VGPRs); each thread then takes `items` pixels.
constexpr int kLifQFwdBlocks = 6 * 256, kLifQBwdBlocks = 4 * 256;

__host__ __device__ constexpr int lifq_ppb(int C) { return NT / (C / 4); }

inline int lifq_items(int64_t npix, int C, int target) {
    const int64_t b1 = (npix + lifq_ppb(C) - 1) / lifq_ppb(C);
    const int64_t it = (b1 + target - 1) / target;
    return (int)(it < 1 ? 1 : it);
}

inline int lifq_grid(int64_t npix, int C, int items) {
    const int64_t per = (int64_t)lifq_ppb(C) * items;
    const int64_t g = (npix + per - 1) / per;
    return (int)(g < 1 ? 1 : g);
}

// OR of a lane value over the Q consecutive lanes of one pixel (Q a power of two <= 8)
template <int Q>
__device__ inline unsigned quad_or(unsigned v) {
#pragma unroll
    for (int o = 1; o < Q; o <<= 1) v |= (unsigned)__shfl_xor((int)v, o, 64);
    return v;
}

// NTH threads per block (NT standalone, NT * 2 as a wavefront task); g: the block's grid (a task's
// block range inside a wavefront launch); each thread takes `items` = ceil(npix / (PPB g.nb)) pixels.
template <int C, int NTH>
__device__ inline int lifq_body_items(int64_t npix, const Grid& g) {
    const int64_t per = (int64_t)(NTH / (C / 4)) * g.nb;
    return (int)((npix + per - 1) / per);
}

// LDS (floats, carved out of the caller's pool: inside a wavefront launch the task kinds share one
// pool) of the quad bodies
template <int C>
constexpr int kLifQFwdLds = 4 * C + 4 * C;  // coef[C], sums[2C] (doubles)
template <int C, bool PRED>
constexpr int kLifQBwdLds = 4 * C + C + (C / 4) * (12 + (PRED ? 10 : 4));  // coef[C], meanv[C], red[Q][NVQ]

template <int C, bool PRED, int NTH>
__device__ void lif_fwd_q_body(const snnflow_lif_fwd_args& a, const Grid g, float* lds) {
    constexpr int Q = C / 4, PPB = NTH / Q;
    static_assert(Q >= 1 && Q <= 8 && (Q & (Q - 1)) == 0, "C = 4, 8, 16, 32");
    LifCoef* const coef = reinterpret_cast<LifCoef*>(lds);
    double* const sums = reinterpret_cast<double*>(lds + 4 * C);
    const int tid = threadIdx.x, q = tid % Q, ps = tid / Q;
    const int64_t HWp = (int64_t)a.H * a.W, npix = (int64_t)a.B * HWp, plane4 = npix * Q;
    const int items = lifq_body_items<C, NTH>(npix, g);
    const float4* y4 = reinterpret_cast<const float4*>(a.y);
    const float4* m4 = reinterpret_cast<const float4*>(a.mem);
    const bool lead = g.bid == 0;
    AccGather<2 * C> gat;
    if (a.n.bn_train) acc_gather_load<2 * C>(a.acc, 2 * C, gat);
    const NeuronRegs nr = load_neuron(a.n, C, lead);
    int64_t p = (int64_t)g.bid * items * PPB + ps;
    int64_t pc = p < npix ? p : npix - 1;  // unconditional 16-B loads
    float4 yv = y4[pc * Q + q], mv = ld4_or_zero(m4, y4, pc * Q + q);
    if (a.n.bn_train) acc_gather_reduce<2 * C>(gat, sums);
    lif_prologue(a.n, nr, sums, C, (double)npix, a.stats, coef, nullptr, lead);
    __syncthreads();
    zero_consumed(a.zero0, a.zero1, a.zero_n, g);
    const bool zr = a.n.zero_reset != 0;
    const LifCoef kc[4] = {coef[4 * q], coef[4 * q + 1], coef[4 * q + 2], coef[4 * q + 3]};
    float4* st4 = reinterpret_cast<float4*>(a.state);
    for (int it = 0; it < items; ++it) {
        const bool act = p < npix;
        const int64_t pn = p + PPB, pcn = pn < npix ? pn : npix - 1;
        float4 yn = yv, mn = mv;
        if (it + 1 < items) {  // next pixel's loads in flight during this one's math
            yn = y4[pcn * Q + q];
            mn = ld4_or_zero(m4, y4, pcn * Q + q);
        }
        const Lif4 o = lif_step4(yv, mv, kc, zr);
        if (act) {
            st4[p * Q + q] = o.mout;
            if (!a.state_spk_skip) st4[plane4 + p * Q + q] = o.s;
        }
        if constexpr (PRED) {
            // the pixel's C spikes as a bit mask on each of its lanes; the 1x1 conv then runs in
            // lane q = o (q = 0 for both outputs at C = 4) in channel order, as one thread per
            // pixel does (bit-identical flows)
            unsigned bits = (o.s.x > 0.f ? 1u : 0u) | (o.s.y > 0.f ? 2u : 0u) | (o.s.z > 0.f ? 4u : 0u) |
                            (o.s.w > 0.f ? 8u : 0u);
            bits = quad_or<Q>(bits << (4 * q));
            const cfloat_ptr pw = as_const(a.pred_w);
            const int64_t b = pc / HWp, hw = pc - b * HWp;
#pragma unroll
            for (int ou = 0; ou < 2; ++ou) {
                if (act && q == (Q >= 2 ? ou : 0)) {
                    float acc = 0.0f;
#pragma unroll
                    for (int c = 0; c < C; ++c) acc = fmaf(pw[ou * C + c], ((bits >> c) & 1u) ? 1.0f : 0.0f, acc);
                    a.flow[(b * 2 + ou) * HWp + hw] = tanhf(acc + a.pred_b[ou]);
                }
            }
        }
        p = pn;
        pc = pcn;
        yv = yn;
        mv = mn;
    }
}

template <int C, bool PRED>
__global__ __launch_bounds__(NT) void k_lif_fwd_q(snnflow_lif_fwd_args a) {
    __shared__ __attribute__((aligned(16))) float pool[kLifQFwdLds<C>];
    lif_fwd_q_body<C, PRED, NT>(a, hw_grid(), pool);
}

template <int C, bool PRED, int NTH>
__device__ void lif_bwd_q_body(const snnflow_lif_bwd_args& a, const Grid gr, float* lds) {
    constexpr int Q = C / 4, PPB = NTH / Q;
    // (g, (y - mean) g, g m') x 4, then [pred: (gpre0 s, gpre1 s) x 4 + gpre0, gpre1] or
    // [no pred: g_mo (1 - s + r) x 4, the membrane-output threshold part of detach=False cells]
    constexpr int NVQ = 12 + (PRED ? 10 : 4);
    static_assert(Q >= 1 && Q <= 8 && (Q & (Q - 1)) == 0, "C = 4, 8, 16, 32");
    static_assert(kLifQBwdLds<C, PRED> == 5 * C + Q * NVQ, "LDS size");
    LifCoef* const coef = reinterpret_cast<LifCoef*>(lds);
    float* const meanv = lds + 4 * C;
    float(*const red)[NVQ] = reinterpret_cast<float(*)[NVQ]>(lds + 5 * C);  // [Q][NVQ] block totals (LDS atomics)
    const int tid = threadIdx.x, q = tid % Q, ps = tid / Q, lane = tid & 63;
    const int64_t HWp = (int64_t)a.H * a.W, npix = (int64_t)a.B * HWp, plane4 = npix * Q;
    const int items = lifq_body_items<C, NTH>(npix, gr);
    LifCoef kci = {0.f, 0.f, 0.f, 0.f};
    float mu = 0.f;
    if (tid < C) {
        kci = lif_coef(a.n, a.stats, C, tid);
        mu = a.stats[tid];
    }
    const float4* y4 = reinterpret_cast<const float4*>(a.y);
    const float4* m4 = reinterpret_cast<const float4*>(a.mem);
    const float4* go4 = reinterpret_cast<const float4*>(a.g_out);
    const float4* gst4 = reinterpret_cast<const float4*>(a.g_state);
    float4* gc4 = reinterpret_cast<float4*>(a.g_cur);
    float4* gm4 = reinterpret_cast<float4*>(a.g_mem);
    const bool mgi = !PRED && a.mem_grad_in && gst4;
    struct Px { float4 y, m, g, gm; float fl[2], gf[2]; };
    auto load = [&](int64_t pp, Px& x) {
        const int64_t pc = pp < npix ? pp : npix - 1;
        const int64_t i = pc * Q + q;
        x.y = y4[i];
        x.m = ld4_or_zero(m4, y4, i);
        x.g = ld4_or_zero(go4, y4, i);
        const float4 t = ld4_or_zero(gst4 ? gst4 + plane4 : nullptr, y4, i);
        if (gst4) x.g = make_float4(x.g.x + t.x, x.g.y + t.y, x.g.z + t.z, x.g.w + t.w);
        x.gm = ld4_or_zero(mgi ? gst4 : nullptr, y4, i);
        x.fl[0] = x.fl[1] = x.gf[0] = x.gf[1] = 0.f;
        if constexpr (PRED) {
            if (a.g_flow) {
                const int64_t b = pc / HWp, hw = pc - b * HWp;
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    x.fl[o] = a.flow[(b * 2 + o) * HWp + hw];
                    x.gf[o] = a.g_flow[b * a.gflow_sb + o * a.gflow_sc + hw];
                }
            }
        }
    };
    int64_t p = (int64_t)gr.bid * items * PPB + ps;
    Px cur;
    load(p, cur);
    if (tid < C) {
        coef[tid] = kci;
        meanv[tid] = mu;
    }
    for (int e = tid; e < Q * NVQ; e += NTH) (&red[0][0])[e] = 0.0f;
    __syncthreads();
    const bool zr = a.n.zero_reset != 0;
    const LifCoef kc[4] = {coef[4 * q], coef[4 * q + 1], coef[4 * q + 2], coef[4 * q + 3]};
    const float mq[4] = {meanv[4 * q], meanv[4 * q + 1], meanv[4 * q + 2], meanv[4 * q + 3]};
    const cfloat_ptr pw = as_const(a.pred_w);
    float v[NVQ];
#pragma unroll
    for (int j = 0; j < NVQ; ++j) v[j] = 0.0f;
    for (int it = 0; it < items; ++it) {
        Px nx = cur;
        if (it + 1 < items) load(p + PPB, nx);
        if (p < npix) {
            float gpre[2] = {0.0f, 0.0f};
            if constexpr (PRED) {
                if (a.g_flow) {
#pragma unroll
                    for (int o = 0; o < 2; ++o) gpre[o] = cur.gf[o] * (1.0f - cur.fl[o] * cur.fl[o]);  // tanh backward
                }
            }
            const float yi[4] = {cur.y.x, cur.y.y, cur.y.z, cur.y.w};
            const float mi[4] = {cur.m.x, cur.m.y, cur.m.z, cur.m.w};
            const float gi[4] = {cur.g.x, cur.g.y, cur.g.z, cur.g.w};
            float go[4], gmo[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = 4 * q + j;
                float g = gi[j];
                if constexpr (PRED) {
                    if (a.g_flow) g = g + (pw[c] * gpre[0] + pw[C + c] * gpre[1]);
                }
                const LifOut o = lif_step(yi[j], mi[j], kc[j], zr);
                float gv = atan_sg(o.v - kc[j].theta) * g;
                if constexpr (!PRED) {
                    if (mgi) {
                        const float gm = j == 0 ? cur.gm.x : (j == 1 ? cur.gm.y : (j == 2 ? cur.gm.z : cur.gm.w));
                        const MemOutGrad d = mem_out_grad(g, gm, mi[j], o, kc[j], zr);
                        gv = d.gv;
                        v[12 + j] += d.gth;
                    }
                }
                go[j] = gv;
                gmo[j] = mem_grad(gv, mi[j], kc[j], zr);
                v[j] += gv;
                v[4 + j] += (yi[j] - mq[j]) * gv;
                v[8 + j] += gv * o.mprime;
                if constexpr (PRED) {
                    v[12 + j] += gpre[0] * o.s;
                    v[16 + j] += gpre[1] * o.s;
                }
            }
            gc4[p * Q + q] = make_float4(go[0], go[1], go[2], go[3]);
            if (gm4) gm4[p * Q + q] = make_float4(gmo[0], gmo[1], gmo[2], gmo[3]);
            if constexpr (PRED) {
                if (q == 0) {
                    v[20] += gpre[0];
                    v[21] += gpre[1];
                }
            }
        }
        p += PPB;
        cur = nx;
    }
    // lanes of equal quad (lane % Q) summed across the wave, the waves' totals through LDS atomics
#pragma unroll
    for (int j = 0; j < NVQ; ++j) {
#pragma unroll
        for (int o = Q; o < 64; o <<= 1) v[j] += __shfl_xor(v[j], o, 64);
    }
    if (lane < Q) {
#pragma unroll
        for (int j = 0; j < NVQ; ++j) atomicAdd(&red[lane][j], v[j]);
    }
    __syncthreads();
    double* acc = acc_shard(a.acc, SNNFLOW_BWD_ACC(C), gr.bid);
    for (int e = tid; e < Q * NVQ; e += NTH) {
        const int qq = e / NVQ, j = e - qq * NVQ;
        if (PRED && j >= 20 && qq != 0) continue;  // the per-pixel prediction-bias sums live in quad 0
        const int k = j < 20 ? (j / 4) * C + 4 * qq + (j & 3) : 5 * C + (j - 20);
        atomicAdd(acc + k, (double)red[qq][j]);
    }
    zero_consumed(a.zero0, a.zero1, a.zero_n, gr);  // last: no load waits behind these stores
}

template <int C, bool PRED>
__global__ __launch_bounds__(NT) void k_lif_bwd_q(snnflow_lif_bwd_args a) {
    __shared__ __attribute__((aligned(16))) float pool[kLifQBwdLds<C, PRED>];
    lif_bwd_q_body<C, PRED, NT>(a, hw_grid(), pool);
}

// Subtract-reset threshold gradient (include/snnflow.h snnflow_lif_theta_subtract): thread per
// float4 of the NHWC tensors, grid-stride (the channel quad of a thread is fixed), per-block
// channel totals through LDS into part[block][C]; k_lif_theta_reduce then sums the blocks' totals
// in block order (fp64) -- no atomics, so the gradient is the same on every run.
template <int C>
__global__ __launch_bounds__(NT) void k_lif_theta_subtract(const float* __restrict__ g_cur, const float* __restrict__ mem,
                                                        const float* __restrict__ thr, int64_t npix, float* part) {
    constexpr int Q = C / 4;
    __shared__ float4 lds[NT];
    const int tid = threadIdx.x, q = tid % Q;
    const float t0 = thr[4 * q], t1 = thr[4 * q + 1], t2 = thr[4 * q + 2], t3 = thr[4 * q + 3];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t n4 = npix * Q, stride = (int64_t)gridDim.x * NT;  // stride % Q == 0 (Q | 256)
    for (int64_t e = (int64_t)blockIdx.x * NT + tid; e < n4; e += stride) {
        const float4 g = reinterpret_cast<const float4*>(g_cur)[e];
        const float4 m = reinterpret_cast<const float4*>(mem)[e];
        acc.x += (m.x - t0 > 0.0f) ? g.x : 0.0f;
        acc.y += (m.y - t1 > 0.0f) ? g.y : 0.0f;
        acc.z += (m.z - t2 > 0.0f) ? g.z : 0.0f;
        acc.w += (m.w - t3 > 0.0f) ? g.w : 0.0f;
    }
    lds[tid] = acc;
    __syncthreads();
    if (tid < C) {
        const int qq = tid / 4, j = tid & 3;
        float s = 0.0f;
        for (int k = qq; k < NT; k += Q) {
            const float4 v = lds[k];
            s += j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
        }
        part[(int64_t)blockIdx.x * C + tid] = s;
    }
}

__global__ __launch_bounds__(64) void k_lif_theta_reduce(const float* __restrict__ part, int nblk, int c,
                                                      float* g_theta) {
    const int ch = threadIdx.x;
    if (ch >= c) return;
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s += (double)part[(int64_t)b * c + ch];
    g_theta[ch] -= (float)s;
}

// BatchNorm backward of one float4 of channels (torch batch_norm_cpu_backward, train):
// dx = ((g - grad_mean) - (y - mean) * k) * invstd * gamma.
struct BnBwdLds { float mean, inv, gm, k, w; };

__device__ inline float4 bn_bwd4(const float4& g, const float4& y, const BnBwdLds* bp) {
    const float gi[4] = {g.x, g.y, g.z, g.w}, yi[4] = {y.x, y.y, y.z, y.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const BnBwdLds c = bp[j];
        const float dx = (yi[j] - c.mean) * c.k;
        o[j] = (((gi[j] - c.gm) - dx) * c.inv) * c.w;
    }
    return make_float4(o[0], o[1], o[2], o[3]);
}

template <int CIN, int C, bool LIF_IN, bool REC, int SPLIT, bool BFG = false>
struct LayerBwdLds {
    // input gradients with the gradient tile and weights split into bf16 parts (mfma_dgrad_bf6):
    // C = 8 with the weight fragments staged in LDS, C = 16 / 32 (BFG) read from global memory
    static constexpr bool BF6 = kMfma<CIN, C> && (C == 8 || BFG);
    static constexpr bool WL = kWlds<CIN, C> && !BF6;
    static constexpr int FR = FragFloats<BF6 && C == 8, C, NT * SPLIT>::v;
    static constexpr int G = BF6 ? (3 * HN * C / 2 + 3) / 4 * 4 : HN * Pad<C>::v;
    static constexpr int WX = WL ? 9 * C * C : FR, WR = REC ? (WL ? 9 * C * C : FR) : 0;
    static constexpr int FLOATS = G + WX + WR;
    static_assert(!BF6 || G >= NT * Pad<CIN>::v, "output staging aliases the gradient tile");
};

// ds_read_b64_tr_b16 pair -> one 16x16x32 bf16 operand: lane (16 g + i) receives column i of 8
// LDS rows (rows 0..3 addressed by lanes 4q + p of its group through r0, rows 4..7 through r1, each
// already offset by 4p columns): 8 consecutive reduction elements of channel i.
typedef short s16x4w __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4w lds_s16x4w;
__device__ inline bf16x8 tr8(const __bf16* r0, const __bf16* r1) {
    const s16x4w v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4w*)(r0));
    const s16x4w v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4w*)(r1));
    const short __attribute__((ext_vector_type(8))) v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}

// Fused weight gradients of a C = 8 LIF-fed layer (snnflow_layer_bwd_args.wslab_*, wavefront
// launches): LDS layout inside the weight-fragment regions, which are free once the input-gradient
// convs are done.  wl_x: X = layer l-1's spikes of the tile [256][8] bf16 (1024 floats), then the
// per-tap results R [c][cin][9] (576 floats) and the tap-8 partials of the 8 waves [8][64];
// wl_r (recurrent cells): the same for the previous-step spikes S.
constexpr int kWgfX = NT * 8 / 2, kWgfR = 8 * 8 * 9, kWgfP = 8 * 64;
constexpr int kWgfFloats = kWgfX + kWgfR + kWgfP;

// Stage of the fused weight gradients, between the input-gradient convs and the store of their
// results (G, the bf16 hi/mid/lo gradient tile with its halo, is still intact):
//   1. the old slab values (accumulate) and the previous-step spikes are loaded;
//   2. barrier (weight fragments dead); X = this pixel's recomputed layer l-1 spikes, S = s_prev;
//   3. barrier; wave w runs tap w over the 8 tile rows (K = 32 pixels each) and row w of tap 8:
//      D[co][ci] += G[q - k][co] X[q][ci] as lo, mid, hi products (exact f32 products: spikes are
//      0/1), A = G through the transposed LDS reads (rows = pixels shifted by the tap), B = X;
//   4. results to R / the tap-8 partials (the caller's barrier completes them).
template <bool REC>
__device__ void fused_wgrad_old(const snnflow_layer_bwd_args& a, const Grid& g, float (&wold)[4]) {
    const int tid = threadIdx.x;
    const bool acc_in = a.wslab_accumulate != 0;
    const bool has_s = REC && a.s_prev != nullptr && a.wslab_rec != nullptr;
    if (acc_in) {
        const float* sf = a.wslab_ff + (int64_t)g.bid * kWgfR;
        wold[0] = sf[tid];
        if (tid + 2 * NT < kWgfR) wold[1] = sf[tid + 2 * NT];
        if constexpr (REC) {
            if (has_s) {
                const float* sr = a.wslab_rec + (int64_t)g.bid * kWgfR;
                wold[2] = sr[tid];
                if (tid + 2 * NT < kWgfR) wold[3] = sr[tid + 2 * NT];
            }
        }
    }
}

template <bool REC>
__device__ void fused_wgrad_stage(const snnflow_layer_bwd_args& a, const float* G, float* wl_x, float* wl_r,
                                  const float (&xsp)[4], const float4& sp, int pt, int ci0) {
    constexpr int C = 8, PART = HN * C;
    const int tid = threadIdx.x;
    const bool has_s = REC && a.s_prev != nullptr && a.wslab_rec != nullptr;
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    __bf16* X = reinterpret_cast<__bf16*>(wl_x);
    __bf16* S = reinterpret_cast<__bf16*>(wl_r);
    const bf16x4 xs = {(__bf16)xsp[0], (__bf16)xsp[1], (__bf16)xsp[2], (__bf16)xsp[3]};
    __syncthreads();  // every wave is done with the staged input-gradient results: the regions are free
    *reinterpret_cast<bf16x4*>(X + pt * C + ci0) = xs;
    if constexpr (REC) {
        if (has_s) *reinterpret_cast<bf16x4*>(S + pt * C + ci0) = bf16x4{(__bf16)sp.x, (__bf16)sp.y, (__bf16)sp.z, (__bf16)sp.w};
    }
    __syncthreads();

    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const __bf16* G3 = reinterpret_cast<const __bf16*>(G);
    const int j0 = 8 * g4 + qq;  // tile column of this lane's first pixel row (the second: + 4)
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc8 = acc, accr = acc, acc8r = acc;
    auto kstep = [&](int tap, int row, f32x4& d, f32x4& dr) {
        const int ky = tap / 3, kx = tap - 3 * ky;
        const int hp = (row + 2 - ky) * HWD + (j0 + 2 - kx);
        const __bf16* ga = G3 + hp * C + 4 * pp;
        const bf16x8 ah = tr8(ga, ga + 4 * C);
        const bf16x8 am = tr8(ga + PART, ga + PART + 4 * C);
        const bf16x8 al = tr8(ga + 2 * PART, ga + 2 * PART + 4 * C);
        const int q = row * TW + j0;
        const __bf16* xb = X + q * C + 4 * pp;
        const bf16x8 b = tr8(xb, xb + 4 * C);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, b, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, b, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b, d, 0, 0, 0);
        if constexpr (REC) {
            if (has_s) {
                const __bf16* sb = S + q * C + 4 * pp;
                const bf16x8 bs = tr8(sb, sb + 4 * C);
                dr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bs, dr, 0, 0, 0);
                dr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bs, dr, 0, 0, 0);
                dr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bs, dr, 0, 0, 0);
            }
        }
    };
#pragma unroll 2
    for (int row = 0; row < TH; ++row) kstep(wv, row, acc, accr);
    kstep(8, wv, acc8, acc8r);
    // lane: D[co = 4 g4 + j][ci = lane & 15]; co, ci < 8 are the layer's
    const int ci = lane & 15;
    if (ci < C && g4 < 2) {
        float* R = wl_x + kWgfX;
        float* P8 = R + kWgfR;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 4 * g4 + j;
            R[(co * C + ci) * 9 + wv] = acc[j];
            P8[wv * 64 + co * C + ci] = acc8[j];
        }
        if constexpr (REC) {
            if (has_s) {
                float* Rr = wl_r + kWgfX;
                float* P8r = Rr + kWgfR;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int co = 4 * g4 + j;
                    Rr[(co * C + ci) * 9 + wv] = accr[j];
                    P8r[wv * 64 + co * C + ci] = acc8r[j];
                }
            }
        }
    }
}

// LDS slot of tile pixel q in the packed [256][16] bf16 x|s tile (32 B per pixel): the transposed reads
// of one 32-lane half-wave fetch pixels j0..j0+3 (lanes 0-15) and j0+8..j0+11 (lanes 16-31), 256 B
// apart -- the same 64 banks; swapping the two 4-pixel halves of every odd 8-pixel group puts the
// second set 128 B further (SQ_LDS_BANK_CONFLICT: 2-way -> none).
__device__ inline int pk_slot(int q) { return SNNFLOW_SWZ ? q ^ (((q >> 3) & 1) << 2) : q; }
// Channel-quad slot of tile pixel q in the packed dgrad staging ([256][8] f32, 32 B per pixel): the
// 16-lane groups of a ds_read_b128 over consecutive pixels would meet pixels 8 apart on one bank set;
// odd 8-pixel groups swap their two quads.
__device__ inline int pk_quad(int q, int quad) { return SNNFLOW_SWZ ? quad ^ ((q >> 3) & 1) : quad; }

// The recurrent conv's results (weight-gradient set, dgrad staging) 16 floats further than a bank-row
// multiple from the feed-forward conv's: lanes n and n + 8 then write different banks.
constexpr int kPkRecOff = SNNFLOW_SWZ ? 16 : 0;

// The recurrent cell's two weight gradients in one matrix-core pass: the tile holds x and s_prev side
// by side ([256 pixels][x 0..7 | s 8..15] bf16 in wl_x), so the B operand's columns 0..7 are x and
// 8..15 are s_prev -- D[co][n] is dW_ff for n < 8 and dW_rec for n >= 8 (the one-conv form leaves
// columns 8..15 unused).  Results: dW_ff's R / tap-8 partials at wl_r, dW_rec's at wl_r + kWgfR + kWgfP.
__device__ void fused_wgrad_stage_pk(const float* G, float* wl_x, float* wl_r, const float (&xsp)[4], const float4& sp,
                                     int pt, int ci0) {
    constexpr int C = 8, PART = HN * C, XS = 16;
    static_assert(FragFloats<true, 8, 2 * NT>::v >= NT * XS / 2 && FragFloats<true, 8, 2 * NT>::v >= 2 * (kWgfR + kWgfP) + kPkRecOff,
                  "packed x|s tile in wl_x, both result sets in wl_r");
    const int tid = threadIdx.x;
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    __bf16* X = reinterpret_cast<__bf16*>(wl_x);
    __syncthreads();  // every wave is done with the staged input-gradient results: the regions are free
    const int ps = pk_slot(pt);
    *reinterpret_cast<bf16x4*>(X + ps * XS + ci0) = bf16x4{(__bf16)xsp[0], (__bf16)xsp[1], (__bf16)xsp[2], (__bf16)xsp[3]};
    *reinterpret_cast<bf16x4*>(X + ps * XS + C + ci0) = bf16x4{(__bf16)sp.x, (__bf16)sp.y, (__bf16)sp.z, (__bf16)sp.w};
    __syncthreads();

    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    const __bf16* G3 = reinterpret_cast<const __bf16*>(G);
    const int j0 = 8 * g4 + qq;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc8 = acc;
    auto kstep = [&](int tap, int row, f32x4& d) {
        const int ky = tap / 3, kx = tap - 3 * ky;
        const int hp = (row + 2 - ky) * HWD + (j0 + 2 - kx);
        const __bf16* ga = G3 + hp * C + 4 * pp;
        const bf16x8 ah = tr8(ga, ga + 4 * C);
        const bf16x8 am = tr8(ga + PART, ga + PART + 4 * C);
        const bf16x8 al = tr8(ga + 2 * PART, ga + 2 * PART + 4 * C);
        const int q = row * TW + j0;
        const bf16x8 b = tr8(X + pk_slot(q) * XS + 4 * pp, X + pk_slot(q + 4) * XS + 4 * pp);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, b, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, b, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b, d, 0, 0, 0);
    };
#pragma unroll 2
    for (int row = 0; row < TH; ++row) kstep(wv, row, acc);
    kstep(8, wv, acc8);
    const int n = lane & 15;
    if (g4 < 2) {  // co = 4 g4 + j < 8
        float* R = wl_r + (n < C ? 0 : kWgfR + kWgfP + kPkRecOff);
        float* P8 = R + kWgfR;
        const int ci = n & 7;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 4 * g4 + j;
            R[(co * C + ci) * 9 + wv] = acc[j];
            P8[wv * 64 + co * C + ci] = acc8[j];
        }
    }
}

// The block's slab rows: element e of [c][cin][9] = R[e] (taps 0..7) or the tap-8 partials of the
// 8 waves summed in wave order; written or added to the old value (fixed order over the steps).
// rx / rr: the R arrays of the two convs (the tap-8 partials follow each).
template <bool REC>
__device__ void fused_wgrad_store(const snnflow_layer_bwd_args& a, const Grid& g, const float* rx,
                                  const float* rr, const float (&wold)[4]) {
    const int tid = threadIdx.x;
    const bool acc_in = a.wslab_accumulate != 0;
    const bool has_s = REC && a.s_prev != nullptr && a.wslab_rec != nullptr;
    auto value = [&](const float* R, int e) {
        const int tap = e % 9;
        if (tap < 8) return R[e];
        const float* P8 = R + kWgfR;
        const int k = e / 9;
        float v = P8[k];
#pragma unroll
        for (int w = 1; w < 8; ++w) v += P8[w * 64 + k];
        return v;
    };
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 2 * NT;
        if (e < kWgfR) {
            a.wslab_ff[(int64_t)g.bid * kWgfR + e] = acc_in ? wold[i] + value(rx, e) : value(rx, e);
            if constexpr (REC) {
                if (a.wslab_rec) {
                    if (has_s) a.wslab_rec[(int64_t)g.bid * kWgfR + e] = acc_in ? wold[2 + i] + value(rr, e) : value(rr, e);
                    else if (!acc_in) a.wslab_rec[(int64_t)g.bid * kWgfR + e] = 0.0f;
                }
            }
        }
    }
}

// Accumulator set of one (conv, thread): item q (tap, co-block of 4, ci-block of VW) and
// pixel group g of the tile, summed over the steps.  Threads [TOFF, TOFF+NTH) of the block
// take part; items x groups fill them (groups reduced in fixed order by flush).
template <int CIN, int C, int NTH, int TOFF>
struct WAcc {
    static constexpr int VW = VecW<CIN>::v;
    static constexpr int Q = 9 * (C / 4) * (CIN / VW);
    static constexpr int GR0 = (Q >= NTH) ? 1 : NTH / Q;
    static constexpr int GR = GR0 > 16 ? 16 : GR0;
    static constexpr int NM = (GR > 1) ? 1 : (Q + NTH - 1) / NTH;
    static constexpr int SCRATCH = (GR > 1) ? GR * Q * 4 * VW : 1;
    float acc[NM][4][VW];
    __device__ void zero() {
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < VW; ++j) acc[m][i][j] = 0.f;
    }
    // Gi: interior G tile [NT][Pad<C>] (HG: the halo G tile [HN][Pad<C>] of the backward task, read at
    // the interior pixels); X: halo input tile [HN][Pad<CIN>]
    template <bool HG = false>
    __device__ void step(const float* Gi, const float* X) {
        constexpr int PC = Pad<C>::v, PX = Pad<CIN>::v;
        const int tid = (int)threadIdx.x - TOFF;
        if (tid < 0 || tid >= NTH) return;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const int q = (GR > 1) ? tid % Q : tid + m * NTH;
            const int g = (GR > 1) ? tid / Q : 0;
            if ((GR > 1) ? (g >= GR) : (q >= Q)) continue;
            const int kidx = q % 9, rest = q / 9, cob = rest % (C / 4), cib = rest / (C / 4);
            const int ky = kidx / 3, kx = kidx % 3;
#pragma unroll 4
            for (int p = g; p < NT; p += GR) {
                const int ty = p / TW, tx = p - ty * TW;
                const int gp = HG ? (ty + 1) * HWD + tx + 1 : p;
                const float4 gv4 = *reinterpret_cast<const float4*>(Gi + gp * PC + cob * 4);
                const float gv[4] = {gv4.x, gv4.y, gv4.z, gv4.w};
                const float* xp = X + ((ty + ky) * HWD + tx + kx) * PX + cib * VW;
                float xv[VW];
                if constexpr (VW == 4) {
                    const float4 v = *reinterpret_cast<const float4*>(xp);
                    xv[0] = v.x; xv[1] = v.y; xv[2] = v.z; xv[3] = v.w;
                } else if constexpr (VW == 2) {
                    const float2 v = *reinterpret_cast<const float2*>(xp);
                    xv[0] = v.x; xv[1] = v.y;
                } else {
                    xv[0] = xp[0];
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < VW; ++j) acc[m][i][j] = fmaf(gv[i], xv[j], acc[m][i][j]);
            }
        }
    }
    // slab element of reduction item e (0 <= e < Q * 4 * VW) of the group-scratch flush
    static __device__ int slab_index(int e) {
        const int qq = e / (4 * VW), ij = e - qq * 4 * VW, i = ij / VW, j = ij - i * VW;
        const int kk = qq % 9, rest = qq / 9, cb = rest % (C / 4), ib = rest / (C / 4);
        return ((cb * 4 + i) * CIN + ib * VW + j) * 9 + kk;
    }
    static constexpr int NOLD = (Q * 4 * VW + NTH - 1) / NTH;  // reduction items per thread
    // flush (GR > 1) with the slab's old values already in registers (old[k]: item tid + k NTH),
    // loaded by the caller long before: the read-modify-write then waits on no global load
    __device__ void flush_prefetched(float* __restrict__ slab, int accumulate, float* scratch, const float (&old)[NOLD]) {
        static_assert(GR > 1, "group-scratch form");
        const int tid = (int)threadIdx.x - TOFF;
        const bool mine = tid >= 0 && tid < NTH;
        const int q = tid % Q, g = tid / Q;
        if (mine && g < GR) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < VW; ++j) scratch[((g * Q + q) * 4 + i) * VW + j] = acc[0][i][j];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NOLD; ++k) {
            const int e = tid + k * NTH;
            if (mine && e < Q * 4 * VW) {
                float sum = 0.f;
                for (int gg = 0; gg < GR; ++gg) sum += scratch[gg * Q * 4 * VW + e];
                slab[slab_index(e)] = accumulate ? old[k] + sum : sum;
            }
        }
    }
    // cross-group reduction in fixed order, then one write (or add) of the block's slab
    __device__ void flush(float* __restrict__ slab, int accumulate, float* scratch) {
        const int tid = (int)threadIdx.x - TOFF;
        const bool mine = tid >= 0 && tid < NTH;
        if constexpr (GR > 1) {
            const int q = tid % Q, g = tid / Q;
            if (mine && g < GR) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < VW; ++j) scratch[((g * Q + q) * 4 + i) * VW + j] = acc[0][i][j];
            }
            __syncthreads();
            for (int e = mine ? tid : Q * 4 * VW; e < Q * 4 * VW; e += NTH) {
                float sum = 0.f;
                for (int gg = 0; gg < GR; ++gg) sum += scratch[gg * Q * 4 * VW + e];
                const int qq = e / (4 * VW), ij = e - qq * 4 * VW, i = ij / VW, j = ij - i * VW;
                const int kk = qq % 9, rest = qq / 9, cb = rest % (C / 4), ib = rest / (C / 4);
                const int idx = ((cb * 4 + i) * CIN + ib * VW + j) * 9 + kk;
                slab[idx] = accumulate ? slab[idx] + sum : sum;
            }
            __syncthreads();
        } else {
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                const int q = tid + m * NTH;
                if (!mine || q >= Q) continue;
                const int kk = q % 9, rest = q / 9, cb = rest % (C / 4), ib = rest / (C / 4);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < VW; ++j) {
                        const int idx = ((cb * 4 + i) * CIN + ib * VW + j) * 9 + kk;
                        slab[idx] = accumulate ? slab[idx] + acc[m][i][j] : acc[m][i][j];
                    }
            }
        }
    }
};

template <int CIN, int C, bool LIF_IN, bool REC, int SPLIT, bool BFG = false, bool WGF = false, bool HWG = false>
__device__ void layer_bwd_body(const snnflow_layer_bwd_args& a, const Grid g, float* lds) {
    using LB = LayerBwdLds<CIN, C, LIF_IN, REC, SPLIT, BFG>;
    static_assert(!HWG || (!LIF_IN && !REC && !kMfma<CIN, C>), "fused head weight gradient: feed-forward head tasks");
    static_assert(!WGF || (LIF_IN && C == 8 && CIN == 8 && SPLIT == 2 && LB::BF6 && LB::FR >= kWgfFloats),
                  "fused weight gradients: C = 8 LIF-fed layers with LDS weight fragments");
    constexpr int NTB = NT * SPLIT;
    constexpr int CI = CIN / SPLIT, CR = C / SPLIT;  // input / recurrent channels per thread group
    static_assert(CI * SPLIT == CIN && CR * SPLIT == C, "channel split");
    static_assert(!LIF_IN || CI % 4 == 0, "LIF backward group: multiple of 4 channels");
    constexpr int PC = Pad<C>::v;
    constexpr bool PF = Prefetch<C, NTB>::on;  // g_cur / y halos held in registers
    constexpr int NVP = LIF_IN ? 3 * CI : 1;
    constexpr int QI = CI / 4 > 0 ? CI / 4 : 1;  // float4s of this group's channels
    float* G = lds;
    [[maybe_unused]] float* wl_x = lds + LB::G;
    [[maybe_unused]] float* wl_r = wl_x + LB::WX;
    __shared__ BnBwdLds bnp[C];
    __shared__ LifCoef pcoef[LIF_IN ? CIN : 1];
    __shared__ float pmean[LIF_IN ? CIN : 1];

    const int tid = threadIdx.x, pt = tid % NT, ty = pt / TW, tx = pt - ty * TW;
    const int part = thread_part(), ci0 = part * CI, cr0 = part * CR;
    const int H = a.H, W = a.W;
    const Tile tl = block_tile(H, W, g);
    const double N = (double)a.B * H * W;
    const float nf = (float)N;
    const int h = tl.h0 + ty, w = tl.w0 + tx;
    const bool in = (h < H) && (w < W);
    const int64_t pix = ((int64_t)tl.b * H + h) * W + w;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    [[maybe_unused]] constexpr bool TR = LIF_IN && CIN == C && SNNFLOW_TRACE_LAYER;
    [[maybe_unused]] constexpr int TK = REC ? 3 : 2;
    TRACE_AT(TR, TK, 0);

    // 1. every global load of the kernel, issued up front (register prefetch; weights for LDS);
    //    the BN-sum replicas first, so that their reduction overlaps the halo loads
    //    (C <= 16; at C = 32 the 12 extra live registers spill: gathered in place there)
    constexpr bool EARLY_G = C <= 16 && !(REC && C == 8 && !SNNFLOW_EARLY_G_REC8);
    // every block needs only the 2C BatchNorm sums (sum g, sum (y - mean) g) of the replicas; the
    // other neuron-gradient sums only block 0 (a third of the loads and of the reduction elsewhere)
    // (C = 32: one gather of all sums -- the second reduction array would take the slot kernel's LDS
    // past two blocks per CU)
    constexpr int NSUM = SNNFLOW_BWD_ACC(C), NBN = (C <= 16 || SNNFLOW_BWD_GATHER32) ? 2 * C : NSUM;
    const bool lead = g.bid == 0;
    constexpr int NL = NSUM - NBN > 0 ? NSUM - NBN : 1;
    AccGather<NBN> gat;
    AccGather<NL> gat_l;
    if constexpr (EARLY_G) {
        acc_gather_load<NBN>(a.acc_in, NSUM, gat);
        if (NBN < NSUM && lead) acc_gather_load<NL>(a.acc_in + NBN, NSUM, gat_l);
    }
    // per-channel parameters, also ahead of the halo loads
    float st_mean = 0.f, st_inv = 0.f, gamma = 0.f;
    if (tid < C) {
        st_mean = a.stats[tid];
        st_inv = a.stats[C + tid];
        gamma = a.n.bn_weight[tid];
    }
    const NeuronGradRegs ngr =
        load_neuron_grad(a.n, a.stats, C, a.ng, a.accumulate, a.has_pred, a.g_pred_w, a.g_pred_b, g.bid == 0);
    // layer l-1's LIF parameters: the raw values loaded here, the coefficients formed after the halo
    // loads are issued (formed here, the compiler waited for these loads before issuing the halo's)
    float praw[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // mean, invstd, gamma, bias, beta, theta
    if constexpr (LIF_IN) {
        const int c = tid < CIN ? tid : 0;
        praw[0] = a.prev_stats[c];
        praw[1] = a.prev_stats[CIN + c];
        praw[2] = a.prev.bn_weight[c];
        praw[3] = a.prev.bn_bias[c];
        praw[4] = a.prev.beta[c];
        praw[5] = a.prev.threshold[c];
    }

    constexpr bool WL = LB::WL, BF6 = LB::BF6, FLDS = BF6 && C == 8;  // FLDS: fragments in LDS
    WStage<WL ? 9 * C * C : 1, NTB> sw_x, sw_r;
    FragStage<FLDS ? C : 8, FLDS ? CIN : 8, FLDS ? NTB : 64> fs_x, fs_r;
    static_assert(!BF6 || PF, "bf16 gradient tile: register-prefetched halo");
    if constexpr (WL) {
        if (a.wt_bwd_ff) sw_x.load(a.wt_fwd_ff);
        if constexpr (REC) {
            if (a.g_state_prev) sw_r.load(a.wt_fwd_rec);
        }
    }
    // C = 8 recurrent cells: both input gradients in one pass (the recurrent conv's fragments in the
    // unused columns 8..15 of the ff conv's B operand): half the input-gradient MFMAs
    constexpr bool PKC = FLDS && REC && CIN == 8 && C == 8;
    [[maybe_unused]] const bool pkr = PKC && a.wt_bwd_ff != nullptr && a.g_state_prev != nullptr;
    if constexpr (FLDS) {
        if constexpr (PKC) {
            if (pkr) fs_x.load2(a.wt_fwd_ff, a.wt_fwd_rec);
            else if (a.wt_bwd_ff) fs_x.load(a.wt_fwd_ff);
            if (!pkr && a.g_state_prev) fs_r.load(a.wt_fwd_rec);
        } else {
            if (a.wt_bwd_ff) fs_x.load(a.wt_fwd_ff);
            if constexpr (REC) {
                if (a.g_state_prev) fs_r.load(a.wt_fwd_rec);
            }
        }
    }
    // fused head weight gradient (ABI 40): its input halo and the slab row's old values are loaded here,
    // with the task's other loads, so that neither is waited on after the BN backward
    using HAF = WAcc<HWG ? CIN : 4, HWG ? C : 4, NTB, 0>;
    constexpr int HXR = HWG ? (HN * CIN + NTB - 1) / NTB : 1;
    [[maybe_unused]] const bool hwg = HWG && a.wslab_ff != nullptr && a.x != nullptr;
    [[maybe_unused]] float hx[HXR], hold[HAF::NOLD];
    if constexpr (HWG) {
        if (hwg) {
            const float* xb = a.x + (int64_t)tl.b * a.xs_b;
#pragma unroll
            for (int i = 0; i < HXR; ++i) {
                const int e = tid + i * NTB;
                const int ci = e / HN, p = e - ci * HN;  // channel-major: the plane reads coalesce
                const int r = p / HWD, cc = p - r * HWD;
                const int hh = tl.h0 + r - 1, ww = tl.w0 + cc - 1;
                hx[i] = (e < HN * CIN && in_image(hh, ww, H, W)) ? xb[ci * a.xs_c + hh * a.xs_h + ww * a.xs_w] : 0.0f;
            }
            const float* srow = a.wslab_ff + (int64_t)g.bid * (C * CIN * 9);
#pragma unroll
            for (int k = 0; k < HAF::NOLD; ++k) {
                const int e = tid + k * NTB;
                hold[k] = (a.wslab_accumulate && e < C * CIN * 9) ? srow[HAF::slab_index(e < C * CIN * 9 ? e : 0)] : 0.0f;
            }
        }
    }
    float4 rg[PF ? Halo4<C, NTB>::R : 1], ry[PF ? Halo4<C, NTB>::R : 1];
    float4 dy[LIF_IN ? QI : 1], dm[LIF_IN ? QI : 1], dg[LIF_IN ? QI : 1];
    if constexpr (PF) {
        halo_load<C, NTB>(a.g_cur, tl, H, W, rg);
        halo_load<C, NTB>(a.y, tl, H, W, ry);
    }
    // layer l-1's inputs of the LIF backward at this thread's pixel; C = 32 loads them only after
    // the input-gradient convs (48 registers fewer across the matrix-core loop)
    constexpr bool LATE_D = C >= 32 || (C == 8 && (REC ? SNNFLOW_LATE_D_REC8 : SNNFLOW_LATE_D_FF8));
    [[maybe_unused]] float wold[4] = {0.f, 0.f, 0.f, 0.f};  // slab rows' old values (e = tid, tid + 512)
    [[maybe_unused]] float4 wsp = z4;                        // previous-step spikes (recurrent conv input)
    [[maybe_unused]] const bool wgf = WGF && a.wslab_ff != nullptr;
    auto load_prev = [&]() {
        if constexpr (LIF_IN) {
            constexpr int Q4 = CIN / 4;
            const int64_t plane4 = (int64_t)a.B * H * W * Q4;
            const float4* py4 = reinterpret_cast<const float4*>(a.prev_y);
            const float4* pm4 = reinterpret_cast<const float4*>(a.prev_mem);
            const float4* pg4 = reinterpret_cast<const float4*>(a.prev_g_state);
            // unconditional 16-B loads (clamped pixel outside the image; results unused there)
            const int64_t pc = ((int64_t)tl.b * H + (h < H ? h : H - 1)) * W + (w < W ? w : W - 1);
            const int64_t base = pc * Q4 + ci0 / 4;
#pragma unroll
            for (int q = 0; q < QI; ++q) {
                dy[q] = py4[base + q];
                dm[q] = ld4_or_zero(pm4, py4, base + q);
                dg[q] = ld4_or_zero(pg4 ? pg4 + plane4 : nullptr, py4, base + q);
            }
        }
        if constexpr (WGF && REC) {  // previous-step spikes of this pixel (recurrent conv input)
            if (wgf && a.s_prev && a.wslab_rec && in) wsp = reinterpret_cast<const float4*>(a.s_prev)[pix * 2 + ci0 / 4];
        }
    };
    if constexpr (!LATE_D) load_prev();


    // 2. per-channel constants; block 0 finishes layer l's neuron gradients and stores the
    //    BN backward coefficients for the deferred weight gradient
    __shared__ double sums[NSUM];
    if constexpr (EARLY_G) {
        acc_gather_reduce<NBN>(gat, sums);
        if (NBN < NSUM && lead) acc_gather_reduce<NL>(gat_l, sums + NBN);  // (block-uniform: barriers inside)
    } else if constexpr (SNNFLOW_BWD_GATHER32) {
        // C = 32: all NTB threads, the reduction scratch in the pool (not live before stage A)
        double* red = reinterpret_cast<double*>(lds);
        acc_gather_pool<NBN, NTB>(a.acc_in, NSUM, sums, red);
        if (NBN < NSUM && lead) acc_gather_pool<NL, NTB>(a.acc_in + NBN, NSUM, sums + NBN, red);
    } else {
        acc_gather<NBN>(a.acc_in, NSUM, sums);
        if (NBN < NSUM && lead) acc_gather<NL>(a.acc_in + NBN, NSUM, sums + NBN);
    }
    neuron_grads(ngr, sums, C, a.ng, a.has_pred, a.g_pred_w, a.g_pred_b, lead);
    if (tid < C) {
        const float mean = st_mean, inv = st_inv;
        BnBwdLds c;
        c.mean = mean;
        c.inv = inv;
        c.w = gamma;
        if (a.n.bn_train) {
            // torch batch_norm_cpu_backward: k = dotp*invstd*invstd/n, grad_mean = sum/n
            c.k = (float)sums[C + tid] * inv * inv / nf;
            c.gm = (float)(sums[tid] / N);
        } else {
            c.k = 0.0f;
            c.gm = 0.0f;
        }
        bnp[tid] = c;
        if (g.bid == 0 && a.bnc_out) {
            a.bnc_out[tid] = c.gm;
            a.bnc_out[C + tid] = c.k;
        }
    }
    if constexpr (LIF_IN) {
        if (tid < CIN) {
            LifCoef pk;  // lif_coef's arithmetic on the raw values
            pk.alpha = praw[1] * praw[2];
            pk.shift = praw[3] - praw[0] * pk.alpha;
            pk.beta = fminf(fmaxf(praw[4], 0.0f), 1.0f);
            pk.theta = praw[5];
            pcoef[tid] = pk;
            pmean[tid] = praw[0];
        }
    }
    __syncthreads();
    TRACE_AT(TR, TK, 1);
    zero_consumed(a.zero0, a.zero1, a.zero_n, g);  // after the gather (vmcnt counts stores)

    // 3. Stage A: BN backward on the halo -> G = dL/dy (pre-BN conv output of layer l)
    if constexpr (PF) {
        constexpr int Q = C / 4;
        static_assert(NTB % Q == 0, "constant channel quad per thread");
        const int qt = tid % Q;
        const BnBwdLds kb[4] = {bnp[4 * qt], bnp[4 * qt + 1], bnp[4 * qt + 2], bnp[4 * qt + 3]};
#pragma unroll
        for (int i = 0; i < Halo4<C, NTB>::R; ++i) {
            const int e = tid + i * NTB;
            if (e < Halo4<C, NTB>::E) {
                const int p = e / Q;
                const int r = p / HWD, cc = p - r * HWD;
                const bool img = in_image(tl.h0 + r - 1, tl.w0 + cc - 1, H, W);
                const float4 gv = img ? bn_bwd4(rg[i], ry[i], kb) : z4;
                if constexpr (BF6) split3_store4(reinterpret_cast<__bf16*>(G) + p * C + 4 * qt, HN * C, gv);
                else *reinterpret_cast<float4*>(G + p * PC + 4 * qt) = gv;
            }
        }
    } else {
        constexpr int Q = C / 4;
        for (int e = tid; e < Halo4<C>::E; e += NTB) {
            const int p = e / Q, q = e - p * Q;
            const int64_t k = halo_idx4<C>(e, tl, H, W);
            float4 out = z4;
            if (k >= 0)
                out = bn_bwd4(reinterpret_cast<const float4*>(a.g_cur)[k], reinterpret_cast<const float4*>(a.y)[k],
                              bnp + 4 * q);
            *reinterpret_cast<float4*>(G + p * PC + 4 * q) = out;
        }
    }
    if constexpr (WL) {
        if (a.wt_bwd_ff) sw_x.store(wl_x);
        if constexpr (REC) {
            if (a.g_state_prev) sw_r.store(wl_r);
        }
    }
    if constexpr (FLDS) {
        if (a.wt_bwd_ff) fs_x.store(reinterpret_cast<__bf16*>(wl_x));
        if constexpr (REC) {
            if (a.g_state_prev && !pkr) fs_r.store(reinterpret_cast<__bf16*>(wl_r));
        }
    }
    __syncthreads();
    TRACE_AT(TR, TK, 2);

    // 4. Stage B: input gradient (dgrad) of ff and rec convolutions (this group's channels)
    float gx[CI];
#pragma unroll
    for (int ci = 0; ci < CI; ++ci) gx[ci] = 0.0f;
    if constexpr (kMfma<CIN, C>) {
        // matrix-core transposed convs over the whole tile (weights in the [tap][cin][c]
        // layout); results come back through LDS aliasing G, one conv at a time
        constexpr int NW = NTB / 64;
        const bool do_x = a.wt_bwd_ff != nullptr;
        const bool do_r = REC && a.g_state_prev != nullptr;
        constexpr int NG = (C >= 32 && BF6) ? 2 : 1;  // C = 32: waves split the output channels too
        MfmaAcc<C, CIN, NW, NG> ax;
        MfmaAcc<C, C, NW, NG> arr;
        const __bf16* g3 = reinterpret_cast<const __bf16*>(G);
        if (do_x) {
            ax.zero();
            if constexpr (FLDS) {
                if (!PROBE_OFF(1)) mfma_dgrad_bf6<C, CIN, NW>(g3, reinterpret_cast<const __bf16*>(wl_x), ax);
            } else if constexpr (BF6) {
                if (!PROBE_OFF(1)) mfma_dgrad_bf6g<C, CIN, NW, NG>(g3, reinterpret_cast<const __bf16*>(a.wd_ff), ax);
            } else {
                if (!PROBE_OFF(1)) mfma_conv3x3<C, CIN, true, NW, NG>(G, WL ? wl_x : a.wt_fwd_ff, ax);
            }
        }
        if constexpr (REC) {
            if (do_r && !pkr) {
                arr.zero();
                if constexpr (FLDS) {
                    if (!PROBE_OFF(1)) mfma_dgrad_bf6<C, C, NW>(g3, reinterpret_cast<const __bf16*>(wl_r), arr);
                } else if constexpr (BF6) {
                    if (!PROBE_OFF(1)) mfma_dgrad_bf6g<C, C, NW, NG>(g3, reinterpret_cast<const __bf16*>(a.wd_rec), arr);
                } else {
                    if (!PROBE_OFF(1)) mfma_conv3x3<C, C, true, NW, NG>(G, WL ? wl_r : a.wt_fwd_rec, arr);
                }
            }
        }
        if constexpr (LATE_D) load_prev();
        __syncthreads();
        // results staged through LDS: the gradient tile G, or (fused weight gradients, which still
        // read G) the weight-fragment regions wl_x.. (free now; the slot pool holds both of them)
        float* const dgo = (WGF && wgf) ? wl_x : G;
        if constexpr (PKC) {
            if (pkr) {  // columns n < 8: gx -> wl_x [NT][8]; n >= 8: the recurrent gradient -> wl_r [NT][8]
                const int lane = tid & 63, n = lane & 15, g4 = lane >> 4;
                const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
                float* out = (n < 8 ? wl_x : wl_r + kPkRecOff) + (n & 3);
#pragma unroll
                for (int mt = 0; mt < MfmaAcc<C, CIN, NW, NG>::MT; ++mt) {
                    const int T = MfmaAcc<C, CIN, NW, NG>::mt0(wv) + mt, row = T >> 1, c0 = (T & 1) * 16;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int q = row * TW + c0 + g4 * 4 + r;
                        out[q * 8 + 4 * pk_quad(q, (n >> 2) & 1)] = ax.v[mt][0][r];
                    }
                }
                __syncthreads();
                const float4 gv4 = *reinterpret_cast<const float4*>(wl_x + pt * 8 + 4 * pk_quad(pt, ci0 >> 2));
                gx[0] = gv4.x; gx[1] = gv4.y; gx[2] = gv4.z; gx[3] = gv4.w;
                if (in) {
                    const int64_t plane = (int64_t)a.B * H * W * C;
                    float* gsp = a.g_state_prev + pix * C + cr0;
                    if (a.zero_mem_half) *reinterpret_cast<float4*>(gsp) = z4;
                    *reinterpret_cast<float4*>(gsp + plane) =
                        *reinterpret_cast<const float4*>(wl_r + kPkRecOff + pt * 8 + 4 * pk_quad(pt, cr0 >> 2));
                }
            }
        }
        if (do_x && !pkr) {
            mfma_store<false>(ax, ax, dgo);
            __syncthreads();
            const float* gl = dgo + pt * Pad<CIN>::v + ci0;
#pragma unroll
            for (int ci = 0; ci < CI; ++ci) gx[ci] = gl[ci];
        }
        if constexpr (REC) {
            if (do_r && !pkr) {
                __syncthreads();
                mfma_store<false>(arr, arr, dgo);
                __syncthreads();
                if (in) {
                    const float* rl = dgo + pt * PC + cr0;
                    const int64_t plane = (int64_t)a.B * H * W * C;
                    float* gsp = a.g_state_prev + pix * C + cr0;
#pragma unroll
                    for (int c = 0; c < CR; c += 4) {
                        if (a.zero_mem_half) *reinterpret_cast<float4*>(gsp + c) = z4;
                        *reinterpret_cast<float4*>(gsp + plane + c) = *reinterpret_cast<const float4*>(rl + c);
                    }
                }
            }
        }
    } else {
        if (!PROBE_OFF(1) && a.wt_bwd_ff) dgrad_acc<C, CIN, CI>(G, a.wt_bwd_ff, ty, tx, ci0, gx);
        if constexpr (REC) {
            if (a.g_state_prev) {
                float gr[CR];
#pragma unroll
                for (int c = 0; c < CR; ++c) gr[c] = 0.0f;
                if (!PROBE_OFF(1)) dgrad_acc<C, C, CR>(G, a.wt_bwd_rec, ty, tx, cr0, gr);
                pin(gr);  // keep the dgrad out of the `in` branch (sinking it there spills SGPRs)
                if (in) {
                    const int64_t plane = (int64_t)a.B * H * W * C;
                    float* gsp = a.g_state_prev + pix * C + cr0;
#pragma unroll
                    for (int c = 0; c < CR; c += 4) {
                        if (a.zero_mem_half) *reinterpret_cast<float4*>(gsp + c) = z4;
                        *reinterpret_cast<float4*>(gsp + plane + c) = make_float4(gr[c], gr[c + 1], gr[c + 2], gr[c + 3]);
                    }
                }
            }
        }
    }

    TRACE_AT(TR, TK, 3);
    // 5. Stage D: LIF backward of layer l-1 on the dgrad result, or the plain input gradient
    if constexpr (LIF_IN) {
        float vd[NVP];
#pragma unroll
        for (int j = 0; j < NVP; ++j) vd[j] = 0.0f;
        [[maybe_unused]] float xsp[4] = {0.f, 0.f, 0.f, 0.f};  // layer l-1's spikes (fused weight gradients)
        if constexpr (WGF) {
            if (wgf) fused_wgrad_old<REC>(a, g, wold);  // in flight during the LIF backward
        }
        if (in && !PROBE_OFF(8)) {
            const bool zr = a.prev.zero_reset != 0;
            float4* gc4 = reinterpret_cast<float4*>(a.prev_g_cur) + pix * (CIN / 4) + ci0 / 4;
            float4* gm4 = a.prev_g_mem ? reinterpret_cast<float4*>(a.prev_g_mem) + pix * (CIN / 4) + ci0 / 4 : nullptr;
#pragma unroll
            for (int q = 0; q < QI; ++q) {
                const float yi[4] = {dy[q].x, dy[q].y, dy[q].z, dy[q].w};
                const float mi[4] = {dm[q].x, dm[q].y, dm[q].z, dm[q].w};
                const float gi[4] = {dg[q].x, dg[q].y, dg[q].z, dg[q].w};
                float go[4], gmo[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int cl = 4 * q + j, ci = ci0 + cl;
                    const float gs = gx[cl] + gi[j];
                    const LifOut o = lif_step(yi[j], mi[j], pcoef[ci], zr);
                    const float gv = atan_sg(o.v - pcoef[ci].theta) * gs;
                    if constexpr (WGF) xsp[cl & 3] = o.s;
                    go[j] = gv;
                    gmo[j] = mem_grad(gv, mi[j], pcoef[ci], zr);
                    vd[cl] = gv;
                    vd[CI + cl] = (yi[j] - pmean[ci]) * gv;
                    vd[2 * CI + cl] = gv * o.mprime;
                }
                gc4[q] = make_float4(go[0], go[1], go[2], go[3]);
                if (gm4) gm4[q] = make_float4(gmo[0], gmo[1], gmo[2], gmo[3]);
            }
        }
        TRACE_AT(TR, TK, 4);
        double* acc = acc_shard(a.acc_out, SNNFLOW_BWD_ACC(CIN), g.bid);
        if (!PROBE_OFF(4))
            block_atomic_sum_parts<NVP, SPLIT>(vd, [acc](int pp, int j) {
                const int k = j / CI, jj = j - k * CI;
                return acc + k * CIN + pp * CI + jj;
            });
        TRACE_AT(TR, TK, 5);
        if constexpr (WGF) {
            if (wgf) {
                if (REC && a.s_prev != nullptr && a.wslab_rec != nullptr) {  // dW_ff and dW_rec in one pass
                    fused_wgrad_stage_pk(G, wl_x, wl_r, xsp, wsp, pt, ci0);
                    __syncthreads();
                    fused_wgrad_store<REC>(a, g, wl_r, wl_r + kWgfR + kWgfP + kPkRecOff, wold);
                } else {
                    fused_wgrad_stage<REC>(a, G, wl_x, wl_r, xsp, wsp, pt, ci0);
                    __syncthreads();
                    fused_wgrad_store<REC>(a, g, wl_x + kWgfX, wl_r + kWgfX, wold);
                }
            }
        }
        TRACE_AT(TR, TK, 6);
    } else {
        if (a.g_x && a.wt_bwd_ff && in) {
            float* gb = a.g_x + (int64_t)tl.b * a.gxs_b + h * a.gxs_h + w * a.gxs_w;
#pragma unroll
            for (int ci = 0; ci < CI; ++ci) gb[(ci0 + ci) * a.gxs_c] = gx[ci];
        }
        if constexpr (HWG) {
            // the head's weight gradient of this step (ABI 40): G (fp32 halo tile, zero outside the image)
            // is intact; the input halo and the accumulators' group scratch go behind it.  The arithmetic
            // of k_wgrad's vector path (WAcc) for one step, added to the block's slab row.
            if (hwg) {
                float* X = lds + LB::G;
#pragma unroll
                for (int i = 0; i < HXR; ++i) {
                    const int e = tid + i * NTB;
                    if (e < HN * CIN) {
                        const int ci = e / HN, p = e - ci * HN;
                        X[p * Pad<CIN>::v + ci] = hx[i];
                    }
                }
                HAF af;
                af.zero();
                __syncthreads();
                af.template step<true>(G, X);
                __syncthreads();  // G and X read: the group scratch of the flush overlays them
                af.flush_prefetched(a.wslab_ff + (int64_t)g.bid * (C * CIN * 9), a.wslab_accumulate, lds, hold);
            }
        }
    }
}

// C = 32 LIF-fed layers: two blocks per CU (<= 128 registers) once the LIF-backward inputs are
// loaded after the input-gradient convs (LATE_D)
template <int CIN, int C, bool LIF_IN, bool REC, int SPLIT, bool BFG = false>
__global__ __launch_bounds__(NT * SPLIT, (C == 32 && LIF_IN && SPLIT == 2) ? SNNFLOW_L32_WAVES : 1)
void k_layer_bwd(snnflow_layer_bwd_args a) {
    __shared__ __attribute__((aligned(16))) float pool[LayerBwdLds<CIN, C, LIF_IN, REC, SPLIT, BFG>::FLOATS];
    layer_bwd_body<CIN, C, LIF_IN, REC, SPLIT, BFG>(a, hw_grid(), pool);
}

// ---------------------------------------------------------------------------
// Deferred weight gradients (snnflow_wgrad): one block per tile loops over the time
// steps of one layer; the next step's loads are issued before the current step's
// arithmetic (register double buffering); per-thread accumulators live across steps
// and the block writes its slab once.
// ---------------------------------------------------------------------------
typedef const __attribute__((address_space(4))) snnflow_wgrad_args* cwgrad_ptr;

// Matrix-core weight gradient of one block (C >= 16, CIN % 16 == 0): per tap,
//   dW_tap[co][ci] += sum_p G[p][co] * X[halo(p, tap)][ci]
// as v_mfma_f32_16x16x4_f32 with M = co (A = G^T from the interior tile), N = ci (B from the
// halo tile), K = 4 tile pixels per MFMA (lane group g takes pixel 4s + g).  The 9 x (C/16) x
// (CIN/16) output tiles of the ff conv [+ the 9 x (C/16)^2 of the recurrent conv] are dealt
// round-robin to the block's NW waves; accumulators live across all time steps.
template <int CIN, int C, bool REC, int NW>
struct WgradMfma {
    static constexpr int MTc = (C + 15) / 16, NTF = (CIN + 15) / 16, NTR = (C + 15) / 16;
    static constexpr int NFF = 9 * MTc * NTF, NREC = REC ? 9 * MTc * NTR : 0, NTOT = NFF + NREC;
    static constexpr int J = (NTOT + NW - 1) / NW;
    static_assert(C % 8 == 0 && CIN % 8 == 0, "MFMA wgrad: 8-channel multiples (C = 8 pads the 16-wide tiles)");
    f32x4 acc[J];
    // wave-uniform tile decode
    int off[J], mt[J], nt[J], tap[J];
    bool rec[J], live[J];
    __device__ void init() {
        const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
#pragma unroll
        for (int j = 0; j < J; ++j) {
            acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int i = wv + NW * j;
            live[j] = i < NTOT;
            rec[j] = i >= NFF;
            const int ii = rec[j] ? i - NFF : i, ntx = rec[j] ? NTR : NTF;
            tap[j] = live[j] ? ii / (MTc * ntx) : 0;
            const int rem = ii - tap[j] * (MTc * ntx);
            mt[j] = live[j] ? rem / ntx : 0;
            nt[j] = live[j] ? rem - mt[j] * ntx : 0;
            off[j] = (tap[j] / 3) * HWD + (tap[j] % 3);
        }
    }
    // Gi: interior G tile [NT][Pad<C>]; X: halo input [HN][Pad<CIN>]; S: halo s_prev [HN][Pad<C>]
    __device__ void step(const float* Gi, const float* X, const float* S, bool has_s) {
        constexpr int PC = Pad<C>::v, PX = Pad<CIN>::v;
        const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
#pragma unroll 8
        for (int s = 0; s < NT / 4; ++s) {
            const int p = 4 * s + g, ty = p / TW, tx = p - ty * TW;
            const int hb = ty * HWD + tx;
            float a[MTc];
#pragma unroll
            for (int q = 0; q < MTc; ++q) a[q] = (q * 16 + m < C) ? Gi[p * PC + q * 16 + m] : 0.0f;
#pragma unroll
            for (int j = 0; j < J; ++j) {
                if (!live[j] || (rec[j] && !has_s)) continue;
                float av = a[0];
#pragma unroll
                for (int q = 1; q < MTc; ++q)
                    if (mt[j] == q) av = a[q];
                const int n = nt[j] * 16 + m;
                float b = 0.0f;  // padded columns: zero (their outputs are not stored)
                if (rec[j]) {
                    if (n < C) b = S[(hb + off[j]) * PC + n];
                } else if (n < CIN) {
                    b = X[(hb + off[j]) * PX + n];
                }
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b, acc[j], 0, 0, 0);
            }
        }
    }
    // C/D layout: rows co = 16 mt + 4 g + r, column ci = 16 nt + (lane & 15); slab [co][ci][tap]
    __device__ void flush(float* __restrict__ slab_ff, float* __restrict__ slab_rec, int accumulate) {
        const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (!live[j] || (rec[j] && !slab_rec)) continue;
            const int ci = nt[j] * 16 + m, cin = rec[j] ? C : CIN;
            if (ci >= cin) continue;
            float* base = rec[j] ? slab_rec : slab_ff;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = mt[j] * 16 + g * 4 + r;
                if (co >= C) continue;
                float* d = base + ((int64_t)co * cin + ci) * 9 + tap[j];
                *d = accumulate ? *d + acc[j][r] : acc[j][r];
            }
        }
    }
};

// own-pixel float4 elements of a C-channel NHWC tile, distributed over NTH threads
template <int CH, int NTH>
struct Own4 {
    static constexpr int Q = CH / 4, E = NT * Q, R = (E + NTH - 1) / NTH;
};

template <int CIN, int C, bool REC, int SPLIT>
__global__ __launch_bounds__(NT * SPLIT) void k_wgrad(snnflow_wgrad_args) {
    constexpr int NTB = NT * SPLIT;
    constexpr int PC = Pad<C>::v, PI_ = Pad<CIN>::v;
    constexpr bool XV = CIN % 4 == 0;  // x may be dense NHWC (register prefetch)
    // ff items on all threads; with a recurrent conv and SPLIT = 2 each conv gets one
    // half of the block (one accumulator set per thread)
    constexpr bool HALVES = REC && SPLIT == 2;
    using AF = WAcc<CIN, C, HALVES ? NT : NTB, 0>;
    using AR = WAcc<C, C, HALVES ? NT : NTB, HALVES ? NT : 0>;
    constexpr bool MF = C >= 16 && CIN % 16 == 0;  // matrix-core path (WgradMfma; at C = 8 the vector path is faster)
    using O = Own4<C, NTB>;
    constexpr int RX = XV ? Halo4<CIN, NTB>::R : 1, RS = REC ? Halo4<C, NTB>::R : 1;
    constexpr int SCR = MF ? 4 : ((REC && AR::SCRATCH > AF::SCRATCH) ? AR::SCRATCH : AF::SCRATCH);
    __shared__ __attribute__((aligned(16))) float Gi[NT * PC];
    __shared__ __attribute__((aligned(16))) float X[HN * PI_];
    __shared__ __attribute__((aligned(16))) float S[REC ? HN * PC : 4];
    __shared__ __attribute__((aligned(16))) float scratch[SCR];
    __shared__ BnBwdLds coef[SNNFLOW_MAX_WGRAD_STEPS][C];

    // the step table stays in the kernarg segment (scalar loads; a dynamically indexed
    // by-value copy would go to scratch)
    const cwgrad_ptr ap = (cwgrad_ptr)__builtin_amdgcn_kernarg_segment_ptr();
    const int tid = threadIdx.x;
    const int H = ap->H, W = ap->W, nsteps = ap->nsteps;
    const Tile tl = block_tile(H, W);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

    // per-step BN backward coefficients of every channel (one round trip for all steps)
    for (int e = tid; e < nsteps * C; e += NTB) {
        const int t = e / C, c = e - t * C;
        const float* st = ap->steps[t].stats;
        const float* bc = ap->steps[t].bnc;
        BnBwdLds k = {0.f, 1.f, 0.f, 0.f, 1.f};  // no BatchNorm: G = g_cur
        if (st) {
            k.mean = st[c];
            k.inv = st[C + c];
            k.gm = bc[c];
            k.k = bc[C + c];
            k.w = ap->bn_weight[c];
        }
        coef[t][c] = k;
    }

    // narrow strided inputs (the head's NCHW event counts): element-wise register prefetch
    constexpr int RXS = XV ? 1 : (HN * CIN + NTB - 1) / NTB;
    // one step's loads in registers, D steps in flight.  D = 3 for the C = 8 feed-forward layers (the
    // deferred head of the wavefront path, 18 registers per step) measured 33.4-35.0 -> 36.2-36.8 us per
    // cfg2 step (profiles/r06/fuse_head_ab.txt): the head's per-step time is not load latency; D = 1.
    struct Pf {
        float4 rg[O::R], ry[O::R], rx[RX], rs[RS];
        float rxs[RXS];
        bool dense, has_s;
    };
    constexpr int D = 1;
    Pf pf[D];
    auto issue = [&](int t, Pf& f) {  // loads of step t into registers
        const float* g = ap->steps[t].g_cur;
        const float* y = ap->steps[t].y;
#pragma unroll
        for (int i = 0; i < O::R; ++i) {
            const int e = tid + i * NTB;
            const int p = e / O::Q, q = e - p * O::Q;
            const int ty = p / TW, tx = p - ty * TW;
            const int h = tl.h0 + ty, w = tl.w0 + tx;
            const bool ok = e < O::E && h < H && w < W;
            const int64_t k = ok ? (((int64_t)tl.b * H + h) * W + w) * O::Q + q : 0;
            f.rg[i] = ok ? reinterpret_cast<const float4*>(g)[k] : z4;
            f.ry[i] = ok ? reinterpret_cast<const float4*>(y)[k] : z4;
        }
        const float* sx = ap->steps[t].x;
        const float* sp = ap->steps[t].s_prev;
        f.dense = false;
        if constexpr (XV)
            f.dense = ap->steps[t].xs_c == 1 && ap->steps[t].xs_w == CIN && ap->steps[t].xs_h == (int64_t)W * CIN &&
                      ap->steps[t].xs_b == (int64_t)H * W * CIN;
        if constexpr (XV) {
            if (f.dense) halo_load<CIN, NTB>(sx, tl, H, W, f.rx);
        } else {
            const auto& st = ap->steps[t];
            const float* xb = sx + (int64_t)tl.b * st.xs_b;
#pragma unroll
            for (int i = 0; i < RXS; ++i) {
                const int e = tid + i * NTB;
                const int ci = e / HN, p = e - ci * HN;  // channel-major: plane reads coalesce
                const int r = p / HWD, cc = p - r * HWD;
                const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
                f.rxs[i] = (e < HN * CIN && in_image(h, w, H, W)) ? xb[ci * st.xs_c + h * st.xs_h + w * st.xs_w] : 0.0f;
            }
        }
        f.has_s = REC && sp != nullptr;
        if constexpr (REC) {
            if (f.has_s) halo_load<C, NTB>(sp, tl, H, W, f.rs);
        }
    };
    // stage step t: G on the tile interior, x and s_prev halos
    auto stage = [&](int t, const Pf& f) {
#pragma unroll
        for (int i = 0; i < O::R; ++i) {
            const int e = tid + i * NTB;
            if (e < O::E) {
                const int p = e / O::Q, q = e - p * O::Q;
                const int ty = p / TW, tx = p - ty * TW;
                const bool img = tl.h0 + ty < H && tl.w0 + tx < W;  // G = 0 outside the image
                *reinterpret_cast<float4*>(Gi + p * PC + 4 * q) = img ? bn_bwd4(f.rg[i], f.ry[i], &coef[t][4 * q]) : z4;
            }
        }
        if constexpr (XV) {
            if (f.dense) halo_store<CIN, NTB>(X, f.rx);
        }
        if constexpr (!XV) {
#pragma unroll
            for (int i = 0; i < RXS; ++i) {
                const int e = tid + i * NTB;
                if (e < HN * CIN) {
                    const int ci = e / HN, p = e - ci * HN;
                    X[p * PI_ + ci] = f.rxs[i];
                }
            }
        } else if (!f.dense) {
            stage_strided<CIN, NTB>(ap->steps[t].x, ap->steps[t].xs_b, ap->steps[t].xs_c, ap->steps[t].xs_h,
                                    ap->steps[t].xs_w, tl, H, W, X);
        }
        if constexpr (REC) {
            if (f.has_s) halo_store<C, NTB>(S, f.rs);
        }
    };

    AF af;
    AR ar;
    WgradMfma<(MF ? CIN : 8), (MF ? C : 8), REC, NTB / 64> am;
    if constexpr (MF) {
        am.init();
    } else {
        af.zero();
        if constexpr (REC) ar.zero();
    }
#pragma unroll
    for (int k = 0; k < D; ++k)
        if (k < nsteps) issue(k, pf[k]);
    __syncthreads();  // coef
    for (int t0 = 0; t0 < nsteps; t0 += D) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const int t = t0 + k;
            if (t >= nsteps) break;
            stage(t, pf[k]);
            const bool has_s_t = pf[k].has_s;
            __syncthreads();
            if (t + D < nsteps) issue(t + D, pf[k]);  // step t+D's loads fly during the next D steps' math
            if constexpr (MF) {
                am.step(Gi, X, S, has_s_t);
            } else {
                af.step(Gi, X);
                if constexpr (REC) {
                    if (has_s_t) ar.step(Gi, S);
                }
            }
            __syncthreads();
        }
    }
    const int64_t blk = blockIdx.x;
    if constexpr (MF) {
        am.flush(ap->slab_ff + blk * (C * CIN * 9), REC ? ap->slab_rec + blk * (C * C * 9) : nullptr, ap->accumulate);
    } else {
        af.flush(ap->slab_ff + blk * (C * CIN * 9), ap->accumulate, scratch);
        if constexpr (REC) ar.flush(ap->slab_rec + blk * (C * C * 9), ap->accumulate, scratch);
    }
}

// ---------------------------------------------------------------------------
// Weight gradients of the C x C layers on the bf16 matrix cores (snnflow_wgrad with
// exact_inputs: the conv inputs -- spikes -- are exact in bf16).  Per tap,
//   dW_tap[co][ci] = sum_p G[p][co] * X[p + tap][ci]
// as v_mfma_f32_16x16x32_bf16 with M = co (A = G^T split into three bf16 parts, so the
// products are the exact f32 products), N = ci (B = X, exact), K = the 32 pixels of one tile
// row (lane group g: pixels 8g..8g+7).  LDS holds G^T [C][260] f32 and X^T / S^T
// [C][10][40] bf16 (channel-major, padded: conflict-free 16-B reads); one 12-element read
// of a halo row gives the B operands of all three kx taps by register shifts.  The output
// tiles (src, ci-tile, ky) x (kx, co-tile) are split over TG wave groups, the 8 tile rows
// over RG = 8 / TG row groups; row groups are summed through LDS in a fixed order at the
// end (deterministic), then one slab write per block.
// ---------------------------------------------------------------------------
template <int C, bool REC>
struct WbGeo {
    static constexpr int MTc = (C + 15) / 16, NTc = (C + 15) / 16;
    static constexpr int BROWS = (REC ? 2 : 1) * NTc * 3;  // (src, ci-tile, ky)
    static constexpr int TPB = 3 * MTc;                     // tiles per B-row: (kx, co-tile)
    static constexpr int NTOT = BROWS * TPB;
    // wave groups over the tiles: <= 9 accumulator tiles per wave up to C = 16, 18 at C = 32
    static constexpr int TG = C <= 16 ? (REC ? 2 : 1) : (REC ? 4 : 2);
    static constexpr int RG = 8 / TG;
    static constexpr int BRW = BROWS / TG;                  // B-rows per wave
    static constexpr int TPW = BRW * TPB;                   // accumulator tiles per wave
    static_assert(BROWS % TG == 0, "B-rows split evenly over the wave groups");
    static constexpr int GS = NT + 4;                       // G^T channel stride (floats)
    static constexpr int XS = 10 * 40 + 8;                  // X^T channel stride (bf16)
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// C = 32 feed-forward weight gradients without the register prefetch of the next step (A/B):
// <= 128 VGPRs, two blocks per CU (66 KB LDS), so the 512-tile grid of cfg2 is one round and the
// other block's math covers a block's loads.
#ifndef SNNFLOW_WG32_PF
#define SNNFLOW_WG32_PF 1
#endif
#ifndef SNNFLOW_WG32_SPLIT
#define SNNFLOW_WG32_SPLIT 1  // C = 32: k_wgrad_bf32 (two blocks per CU) for feed-forward layers (2: recurrent too)
#endif
template <int C, bool REC>
constexpr bool kWgPf = !(C == 32 && !REC && !SNNFLOW_WG32_PF);

template <int C, bool REC>
__global__ __launch_bounds__(NT * 2, (kWgPf<C, REC> ? 1 : 4)) void k_wgrad_bf(snnflow_wgrad_args) {
    using Gm = WbGeo<C, REC>;
    constexpr bool PF = kWgPf<C, REC>;
    constexpr int NTB = NT * 2, NW = NTB / 64, Q = C / 4;
    constexpr int RX = Halo4<C, NTB>::R;
    using O = Own4<C, NTB>;
    static_assert(NW == 8, "8 waves");
    // one pool for G^T, X^T, S^T: the row-group reduction at the end aliases all of it
    // (separate __shared__ arrays are not guaranteed to be contiguous)
    constexpr int GF = C * Gm::GS, XF = C * Gm::XS / 2, SF = REC ? C * Gm::XS / 2 : 4;
    constexpr int RF = Gm::TG * Gm::TPW * 256;
    __shared__ __attribute__((aligned(16))) float pool[(GF + XF + SF > RF ? GF + XF + SF : RF)];
    float* const Gt = pool;
    unsigned short* const Xt = reinterpret_cast<unsigned short*>(pool + GF);
    unsigned short* const St = reinterpret_cast<unsigned short*>(pool + GF + XF);
    __shared__ BnBwdLds coef[SNNFLOW_MAX_WGRAD_STEPS][C];

    const cwgrad_ptr ap = (cwgrad_ptr)__builtin_amdgcn_kernarg_segment_ptr();
    const int tid = threadIdx.x, lane = tid & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), tg = wv % Gm::TG, rg = wv / Gm::TG;
    const int H = ap->H, W = ap->W, nsteps = ap->nsteps;
    const Tile tl = block_tile(H, W);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

    for (int e = tid; e < nsteps * C; e += NTB) {
        const int t = e / C, c = e - t * C;
        const float* st = ap->steps[t].stats;
        const float* bc = ap->steps[t].bnc;
        BnBwdLds k = {0.f, 1.f, 0.f, 0.f, 1.f};
        if (st) {
            k.mean = st[c];
            k.inv = st[C + c];
            k.gm = bc[c];
            k.k = bc[C + c];
            k.w = ap->bn_weight[c];
        }
        coef[t][c] = k;
    }

    float4 rg4[O::R], ry4[O::R], rx[RX], rs[REC ? RX : 1];
    unsigned rxb[RX], rsb[REC ? RX : 1];  // x / s_prev as spike bit-plane words (ABI 39)
    bool dense = false, has_s = false, xbits = false, sbits = false;
    auto issue = [&](int t) {
        const float* gp = ap->steps[t].g_cur;
        const float* yp = ap->steps[t].y;
#pragma unroll
        for (int i = 0; i < O::R; ++i) {
            const int e = tid + i * NTB;
            const int p = e / Q, q = e - p * Q;
            const int ty = p / TW, tx = p - ty * TW;
            const int h = tl.h0 + ty, w = tl.w0 + tx;
            const bool ok = e < O::E && h < H && w < W;
            const int64_t k = ok ? (((int64_t)tl.b * H + h) * W + w) * Q + q : 0;
            rg4[i] = ok ? reinterpret_cast<const float4*>(gp)[k] : z4;
            ry4[i] = ok ? reinterpret_cast<const float4*>(yp)[k] : z4;
        }
        const auto& sp = ap->steps[t];
        xbits = sp.x_bits != nullptr;
        dense = xbits || (sp.xs_c == 1 && sp.xs_w == C && sp.xs_h == (int64_t)W * C && sp.xs_b == (int64_t)H * W * C);
        if (xbits) halo_load_bits<C, NTB>(sp.x_bits, tl, H, W, rxb);
        else if (dense) halo_load<C, NTB>(sp.x, tl, H, W, rx);
        sbits = REC && sp.s_prev_bits != nullptr;
        has_s = REC && (sp.s_prev != nullptr || sbits);
        if constexpr (REC) {
            if (sbits) halo_load_bits<C, NTB>(sp.s_prev_bits, tl, H, W, rsb);
            else if (has_s) halo_load<C, NTB>(sp.s_prev, tl, H, W, rs);
        }
    };
    // halo float4 element (pixel p, quad q) -> 4 bf16 of the channel-major tile
    auto put_halo = [&](unsigned short* T, int e, const float4& v) {
        const int p = e / Q, q = e - p * Q;
        const int hr = p / HWD, hc = p - hr * HWD;
        unsigned short* d = T + (4 * q) * Gm::XS + hr * 40 + hc;
        d[0] = __builtin_bit_cast(unsigned short, (__bf16)v.x);
        d[Gm::XS] = __builtin_bit_cast(unsigned short, (__bf16)v.y);
        d[2 * Gm::XS] = __builtin_bit_cast(unsigned short, (__bf16)v.z);
        d[3 * Gm::XS] = __builtin_bit_cast(unsigned short, (__bf16)v.w);
    };

    f32x4 acc[Gm::TPW];
#pragma unroll
    for (int j = 0; j < Gm::TPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if constexpr (PF) issue(0);
    __syncthreads();  // coef
    for (int t = 0; t < nsteps; ++t) {
        if constexpr (!PF) issue(t);
        // stage step t: G^T (BN backward of g_cur, zero outside the image), X^T, S^T
#pragma unroll
        for (int i = 0; i < O::R; ++i) {
            const int e = tid + i * NTB;
            if (e < O::E) {
                const int p = e / Q, q = e - p * Q;
                const int ty = p / TW, tx = p - ty * TW;
                const bool img = tl.h0 + ty < H && tl.w0 + tx < W;
                const float4 gv = img ? bn_bwd4(rg4[i], ry4[i], &coef[t][4 * q]) : z4;
                float* d = Gt + (4 * q) * Gm::GS + p;
                d[0] = gv.x;
                d[Gm::GS] = gv.y;
                d[2 * Gm::GS] = gv.z;
                d[3 * Gm::GS] = gv.w;
            }
        }
        const bool dense_t = dense, has_s_t = has_s, xbits_t = xbits, sbits_t = sbits;
        if (xbits_t) {
#pragma unroll
            for (int i = 0; i < RX; ++i) {
                const int e = tid + i * NTB;
                if (e < Halo4<C, NTB>::E) put_halo(Xt, e, spk_quad<C>(rxb[i], e % Q));
            }
        } else if (dense_t) {
#pragma unroll
            for (int i = 0; i < RX; ++i) {
                const int e = tid + i * NTB;
                if (e < Halo4<C, NTB>::E) put_halo(Xt, e, rx[i]);
            }
        } else {  // strided input: element-wise gather (not the engine's path)
            const auto& sp = ap->steps[t];
            for (int e = tid; e < HN * C; e += NTB) {
                const int p = e / C, c = e - p * C;
                const int hr = p / HWD, hc = p - hr * HWD;
                const int h = tl.h0 + hr - 1, w = tl.w0 + hc - 1;
                const float v = in_image(h, w, H, W) ? sp.x[tl.b * sp.xs_b + c * sp.xs_c + h * sp.xs_h + w * sp.xs_w] : 0.f;
                Xt[c * Gm::XS + hr * 40 + hc] = __builtin_bit_cast(unsigned short, (__bf16)v);
            }
        }
        if constexpr (REC) {
            if (sbits_t) {
#pragma unroll
                for (int i = 0; i < RX; ++i) {
                    const int e = tid + i * NTB;
                    if (e < Halo4<C, NTB>::E) put_halo(St, e, spk_quad<C>(rsb[i], e % Q));
                }
            } else if (has_s_t) {
#pragma unroll
                for (int i = 0; i < RX; ++i) {
                    const int e = tid + i * NTB;
                    if (e < Halo4<C, NTB>::E) put_halo(St, e, rs[i]);
                }
            }
        }
        __syncthreads();
        if constexpr (PF) {
            if (t + 1 < nsteps) issue(t + 1);  // next step's loads fly during this step's math
        }

        // compute: this wave's tile rows r = rg, rg + RG, ...
#pragma unroll
        for (int rr = 0; rr < Gm::TG; ++rr) {
            const int r = rg + rr * Gm::RG;
            bf16x8 ah[Gm::MTc], am[Gm::MTc], al[Gm::MTc];
#pragma unroll
            for (int mt = 0; mt < Gm::MTc; ++mt) {
                const int co = mt * 16 + m;
                float a8[8];
                if (co < C) {
                    const float* src = Gt + co * Gm::GS + r * TW + 8 * g;
                    const float4 u = *reinterpret_cast<const float4*>(src), v = *reinterpret_cast<const float4*>(src + 4);
                    a8[0] = u.x; a8[1] = u.y; a8[2] = u.z; a8[3] = u.w; a8[4] = v.x; a8[5] = v.y; a8[6] = v.z; a8[7] = v.w;
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) a8[j] = 0.f;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const __bf16 h = (__bf16)a8[j];
                    const float r1 = a8[j] - (float)h;
                    const __bf16 md = (__bf16)r1;
                    ah[mt][j] = h;
                    am[mt][j] = md;
                    al[mt][j] = (__bf16)(r1 - (float)md);
                }
            }
#pragma unroll
            for (int k = 0; k < Gm::BRW; ++k) {
                const int br = tg * Gm::BRW + k;  // (src, ci-tile, ky), ky fastest
                const int ky = br % 3, nt = (br / 3) % Gm::NTc, src = br / (3 * Gm::NTc);
                if (src == 1 && !has_s_t) continue;
                const int ci = nt * 16 + m;
                unsigned int w6[6] = {0u, 0u, 0u, 0u, 0u, 0u};
                if (ci < C) {
                    const unsigned short* T = (src == 0 ? Xt : St) + ci * Gm::XS + (r + ky) * 40 + 8 * g;
                    const u32x4 u = *reinterpret_cast<const u32x4*>(T);
                    const uint2 v = *reinterpret_cast<const uint2*>(T + 8);
                    w6[0] = u.x; w6[1] = u.y; w6[2] = u.z; w6[3] = u.w; w6[4] = v.x; w6[5] = v.y;
                }
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    u32x4 bw;
                    if (kx == 0) bw = u32x4{w6[0], w6[1], w6[2], w6[3]};
                    else if (kx == 2) bw = u32x4{w6[1], w6[2], w6[3], w6[4]};
                    else bw = u32x4{__builtin_amdgcn_alignbit(w6[1], w6[0], 16), __builtin_amdgcn_alignbit(w6[2], w6[1], 16),
                                    __builtin_amdgcn_alignbit(w6[3], w6[2], 16), __builtin_amdgcn_alignbit(w6[4], w6[3], 16)};
                    const bf16x8 b = __builtin_bit_cast(bf16x8, bw);
#pragma unroll
                    for (int mt = 0; mt < Gm::MTc; ++mt) {
                        f32x4& d = acc[k * Gm::TPB + kx * Gm::MTc + mt];
                        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[mt], b, d, 0, 0, 0);
                        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[mt], b, d, 0, 0, 0);
                        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], b, d, 0, 0, 0);
                    }
                }
            }
        }
        __syncthreads();
    }

    // row groups 1..RG-1 add into row group 0 through LDS (fixed order), aliasing Gt/Xt/St
    float* red = pool;  // [TG][TPW][64][4] floats (RF)
#pragma unroll 1
    for (int q = 1; q < Gm::RG; ++q) {
        if (rg == q) {
#pragma unroll
            for (int j = 0; j < Gm::TPW; ++j)
                *reinterpret_cast<f32x4*>(red + ((tg * Gm::TPW + j) * 64 + lane) * 4) = acc[j];
        }
        __syncthreads();
        if (rg == 0) {
#pragma unroll
            for (int j = 0; j < Gm::TPW; ++j) acc[j] = acc[j] + *reinterpret_cast<const f32x4*>(red + ((tg * Gm::TPW + j) * 64 + lane) * 4);
        }
        __syncthreads();
    }
    if (rg != 0) return;
    const int64_t blk = blockIdx.x;
    const int accumulate = ap->accumulate;
#pragma unroll
    for (int k = 0; k < Gm::BRW; ++k) {
        const int br = tg * Gm::BRW + k;
        const int ky = br % 3, nt = (br / 3) % Gm::NTc, src = br / (3 * Gm::NTc);
        float* slab = (src == 0 ? ap->slab_ff : ap->slab_rec) + blk * (C * C * 9);
        const int ci = nt * 16 + m;
        if (ci >= C) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int mt = 0; mt < Gm::MTc; ++mt) {
                const f32x4 v = acc[k * Gm::TPB + kx * Gm::MTc + mt];
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) {
                    const int co = mt * 16 + 4 * g + r4;
                    if (co >= C) continue;
                    float* d = slab + ((int64_t)co * C + ci) * 9 + ky * 3 + kx;
                    *d = accumulate ? *d + v[r4] : v[r4];
                }
            }
    }
}

// C = 32 weight gradients at two blocks per CU (k_wgrad_bf<32> needs 212-244 VGPRs, one block per
// CU, so the 512-tile grid of cfg2 took two rounds).  Same arithmetic and slab layout as
// k_wgrad_bf; what changes is the split of the work and the staging:
//   * wave w: output tiles of (ci-tile nt = w & 1, co-tile mt = (w >> 1) & 1) -- all 3 x 3 taps,
//     per source 9 accumulator tiles (36 VGPRs) and ONE co-tile's A fragments (hi/mid/lo, 12
//     VGPRs) -- over the tile rows r = (w >> 2) + 2 i (two row groups, summed in LDS at the end);
//   * no next-step loads held in registers: each step's G / y / x loads are issued and stored to LDS
//     in batches (the other resident block's math covers them);
//   * recurrent cells stage S into the X buffer after the X pass (one X buffer: G^T 33 KB + X^T 26 KB
//     + BN coefficients 20 KB = 80 KB of LDS, two blocks per CU; <= 128 VGPRs).
// ---------------------------------------------------------------------------
// A lane's 36 slab elements of one C = 32 weight-gradient tile pair (rows co0 .. co0+3, column ci, the
// 9 taps; v(j) gives tap j's four values): written, or added to the old values -- every old value is
// loaded before the first add (a conditional load per element made the compiler wait 36 round trips).
template <typename F>
__device__ inline void slab_rmw_36(float* slab, int co0, int ci, int accumulate, F&& v) {
    constexpr int C = 32;
    float old[9][4];
    if (accumulate) {
#pragma unroll
        for (int j = 0; j < 9; ++j)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) old[j][r4] = slab[((int64_t)(co0 + r4) * C + ci) * 9 + j];
    } else {
#pragma unroll
        for (int j = 0; j < 9; ++j)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) old[j][r4] = 0.0f;
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        const f32x4 x = v(j);
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) slab[((int64_t)(co0 + r4) * C + ci) * 9 + j] = accumulate ? old[j][r4] + x[r4] : x[r4];
    }
}

template <bool REC>
__global__ __launch_bounds__(NT * 2, 4) void k_wgrad_bf32(snnflow_wgrad_args) {
    constexpr int C = 32, NTB = NT * 2, Q = C / 4;
    constexpr int GS = NT + 4, XS = 10 * 40 + 8;
    constexpr int RX = Halo4<C, NTB>::R;
    using O = Own4<C, NTB>;
    constexpr int NS = REC ? 2 : 1;      // sources: x (ff conv), s_prev (rec conv)
    constexpr int GF = C * GS, XF = C * XS / 2;
    constexpr int RF = 4 * 9 * 256;      // one source's row-group exchange [4 tg][9][64][4]
    static_assert(RF <= GF + XF, "exchange fits the staging pool");
    __shared__ __attribute__((aligned(16))) float pool[GF + XF];
    float* const Gt = pool;
    unsigned short* const Xt = reinterpret_cast<unsigned short*>(pool + GF);
    __shared__ BnBwdLds coef[SNNFLOW_MAX_WGRAD_STEPS][C];

    const cwgrad_ptr ap = (cwgrad_ptr)__builtin_amdgcn_kernarg_segment_ptr();
    const int tid = threadIdx.x, lane = tid & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nt = wv & 1, mt = (wv >> 1) & 1, rg = wv >> 2;
    const int H = ap->H, W = ap->W, nsteps = ap->nsteps;
    const Tile tl = block_tile(H, W);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

    for (int e = tid; e < nsteps * C; e += NTB) {
        const int t = e / C, c = e - t * C;
        const float* st = ap->steps[t].stats;
        const float* bc = ap->steps[t].bnc;
        BnBwdLds k = {0.f, 1.f, 0.f, 0.f, 1.f};
        if (st) {
            k.mean = st[c];
            k.inv = st[C + c];
            k.gm = bc[c];
            k.k = bc[C + c];
            k.w = ap->bn_weight[c];
        }
        coef[t][c] = k;
    }

    // halo float4 element (pixel p, quad q) -> 4 bf16 of the channel-major tile
    auto put_halo = [&](int e, const float4& v) {
        const int p = e / Q, q = e - p * Q;
        const int hr = p / HWD, hc = p - hr * HWD;
        unsigned short* d = Xt + (4 * q) * XS + hr * 40 + hc;
        d[0] = __builtin_bit_cast(unsigned short, (__bf16)v.x);
        d[XS] = __builtin_bit_cast(unsigned short, (__bf16)v.y);
        d[2 * XS] = __builtin_bit_cast(unsigned short, (__bf16)v.z);
        d[3 * XS] = __builtin_bit_cast(unsigned short, (__bf16)v.w);
    };
    // the conv input of step t (x or s_prev) into X^T: dense NHWC halo, or an element-wise gather
    auto stage_x = [&](const float* src, int64_t sb, int64_t sc, int64_t sh, int64_t sw, bool dense,
                       const uint8_t* bits) {
        if (bits) {  // spike bit plane (ABI 39): one word per element, all loads in flight at once
            unsigned rb[RX];
            halo_load_bits<C, NTB>(bits, tl, H, W, rb);
#pragma unroll
            for (int i = 0; i < RX; ++i) {
                const int e = tid + i * NTB;
                if (e < Halo4<C, NTB>::E) put_halo(e, spk_quad<C>(rb[i], e % Q));
            }
        } else if (dense) {  // two batches of loads (12 VGPRs each: the accumulators stay live)
            constexpr int RH = (RX + 1) / 2;
#pragma unroll
            for (int h2 = 0; h2 < RX; h2 += RH) {
                float4 rx[RH];
#pragma unroll
                for (int i = 0; i < RH; ++i) {
                    const int e = tid + (h2 + i) * NTB;
                    const int64_t k = (h2 + i) < RX && e < Halo4<C, NTB>::E ? halo_idx4<C>(e, tl, H, W) : -1;
                    rx[i] = k >= 0 ? reinterpret_cast<const float4*>(src)[k] : z4;
                }
#pragma unroll
                for (int i = 0; i < RH; ++i) {
                    const int e = tid + (h2 + i) * NTB;
                    if ((h2 + i) < RX && e < Halo4<C, NTB>::E) put_halo(e, rx[i]);
                }
            }
        } else {
            for (int e = tid; e < HN * C; e += NTB) {
                const int p = e / C, c = e - p * C;
                const int hr = p / HWD, hc = p - hr * HWD;
                const int h = tl.h0 + hr - 1, w = tl.w0 + hc - 1;
                const float v = in_image(h, w, H, W) ? src[tl.b * sb + c * sc + h * sh + w * sw] : 0.f;
                Xt[c * XS + hr * 40 + hc] = __builtin_bit_cast(unsigned short, (__bf16)v);
            }
        }
    };

    f32x4 acc[NS][9];
#pragma unroll
    for (int sidx = 0; sidx < NS; ++sidx)
#pragma unroll
        for (int j = 0; j < 9; ++j) acc[sidx][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // one source's MFMAs of the staged step: rows r = rg, rg + 2, ..., 9 taps of (nt, mt)
    auto compute = [&](f32x4 (&d)[9]) {
#pragma unroll 1
        for (int r = rg; r < TH; r += 2) {
            bf16x8 ah, am, al;
            {
                const int co = mt * 16 + m;
                const float* src = Gt + co * GS + r * TW + 8 * g;
                const float4 u = *reinterpret_cast<const float4*>(src), v = *reinterpret_cast<const float4*>(src + 4);
                const float a8[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const __bf16 h = (__bf16)a8[j];
                    const float r1 = a8[j] - (float)h;
                    const __bf16 md = (__bf16)r1;
                    ah[j] = h;
                    am[j] = md;
                    al[j] = (__bf16)(r1 - (float)md);
                }
            }
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const unsigned short* T = Xt + (nt * 16 + m) * XS + (r + ky) * 40 + 8 * g;
                const u32x4 u = *reinterpret_cast<const u32x4*>(T);
                const uint2 v = *reinterpret_cast<const uint2*>(T + 8);
                const unsigned int w6[5] = {u.x, u.y, u.z, u.w, v.x};
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    u32x4 bw;
                    if (kx == 0) bw = u32x4{w6[0], w6[1], w6[2], w6[3]};
                    else if (kx == 2) bw = u32x4{w6[1], w6[2], w6[3], w6[4]};
                    else bw = u32x4{__builtin_amdgcn_alignbit(w6[1], w6[0], 16), __builtin_amdgcn_alignbit(w6[2], w6[1], 16),
                                    __builtin_amdgcn_alignbit(w6[3], w6[2], 16), __builtin_amdgcn_alignbit(w6[4], w6[3], 16)};
                    const bf16x8 b = __builtin_bit_cast(bf16x8, bw);
                    f32x4& o = d[ky * 3 + kx];
                    o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, b, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, b, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b, o, 0, 0, 0);
                }
            }
        }
    };

    __syncthreads();  // coef
    for (int t = 0; t < nsteps; ++t) {
        const auto& sp = ap->steps[t];
        // G^T = BN backward of g_cur (zero outside the image), two batches of loads
#pragma unroll
        for (int h2 = 0; h2 < O::R; h2 += 2) {
            float4 rg4[2], ry4[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int e = tid + (h2 + i) * NTB;
                const int p = e / Q, q = e - p * Q;
                const int ty = p / TW, tx = p - ty * TW;
                const int h = tl.h0 + ty, w = tl.w0 + tx;
                const bool ok = e < O::E && h < H && w < W;
                const int64_t k = ok ? (((int64_t)tl.b * H + h) * W + w) * Q + q : 0;
                rg4[i] = ok ? reinterpret_cast<const float4*>(sp.g_cur)[k] : z4;
                ry4[i] = ok ? reinterpret_cast<const float4*>(sp.y)[k] : z4;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int e = tid + (h2 + i) * NTB;
                if (e < O::E) {
                    const int p = e / Q, q = e - p * Q;
                    const int ty = p / TW, tx = p - ty * TW;
                    const bool img = tl.h0 + ty < H && tl.w0 + tx < W;
                    const float4 gv = img ? bn_bwd4(rg4[i], ry4[i], &coef[t][4 * q]) : z4;
                    float* d = Gt + (4 * q) * GS + p;
                    d[0] = gv.x;
                    d[GS] = gv.y;
                    d[2 * GS] = gv.z;
                    d[3 * GS] = gv.w;
                }
            }
        }
        const bool dense = sp.xs_c == 1 && sp.xs_w == C && sp.xs_h == (int64_t)W * C && sp.xs_b == (int64_t)H * W * C;
        stage_x(sp.x, sp.xs_b, sp.xs_c, sp.xs_h, sp.xs_w, dense, sp.x_bits);
        __syncthreads();
        compute(acc[0]);
        if constexpr (REC) {
            if (sp.s_prev != nullptr || sp.s_prev_bits != nullptr) {
                __syncthreads();  // X^T reads done
                stage_x(sp.s_prev, 0, 0, 0, 0, true, sp.s_prev_bits);
                __syncthreads();
                compute(acc[NS - 1]);
            }
        }
        __syncthreads();  // before the next step overwrites the tiles
    }

    // row group 1 adds into row group 0 through LDS (fixed order), one source at a time
    const int64_t blk = blockIdx.x;
    const int accumulate = ap->accumulate;
    float* red = pool;
    const int tg = wv & 3;
#pragma unroll
    for (int sidx = 0; sidx < NS; ++sidx) {
        if (rg == 1) {
#pragma unroll
            for (int j = 0; j < 9; ++j) *reinterpret_cast<f32x4*>(red + ((tg * 9 + j) * 64 + lane) * 4) = acc[sidx][j];
        }
        __syncthreads();
        if (rg == 0) {
            float* slab = (sidx == 0 ? ap->slab_ff : ap->slab_rec) + blk * (C * C * 9);
            const int ci = nt * 16 + m;
            slab_rmw_36(slab, mt * 16 + 4 * g, ci, accumulate, [&](int j) {
                return acc[sidx][j] + *reinterpret_cast<const f32x4*>(red + ((tg * 9 + j) * 64 + lane) * 4);
            });
        }
        __syncthreads();
    }
}

// C = 32 weight gradients from spike bit planes (ABI 39: the deferred weight gradients of the
// wavefront path).  k_wgrad_bf32's arithmetic, slab layout and wave split (wave w: ci-tile w & 1, co-tile
// (w >> 1) & 1, tile rows (w >> 2) + 2 i, all 9 taps), with
//   * the conv input of a step as one 32-bit word per halo pixel (1.4 KB per tile instead of 44 KB of
//     fp32 spikes), expanded to the channel-major bf16 X^T tile by the thread of that pixel;
//   * the next step's loads -- g_cur and y of the tile (8 float4 per thread) and the halo word -- issued
//     right after this step's tiles are staged, so they fly during this step's matrix-core work
//     (k_wgrad_bf32 loads each step after the previous one's MFMAs: its fp32 input halo would not fit
//     beside a prefetch in 128 registers);
//   * a recurrent layer's two convs as two block sets (source 0: x -> slab_ff; 1: s_prev -> slab_rec), each
//     block one source with 36 accumulator registers per wave like a feed-forward layer (k_wgrad_bf<32,
//     true> holds both: 256 registers, one block per CU).  Block b: XCD b % 8, source (b / 8) & 1, tile
//     (b % 8) + 8 (b / 16): the two sources of a tile run on one XCD at about the same time, so the second
//     read of G's inputs is an L2 hit.
// A step whose input has no bit plane (s_prev at t = 0: the caller's initial state) stages the fp32 plane;
// without either it adds nothing.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT * 2, 4) void k_wgrad_b32(snnflow_wgrad_args) {
    constexpr int C = 32, NTB = NT * 2, Q = C / 4;
    constexpr int GS = NT + 4, XS = 10 * 40 + 8;
    using O = Own4<C, NTB>;
    constexpr int GF = C * GS, XF = C * XS / 2;
    constexpr int RF = 4 * 9 * 256;  // one source's row-group exchange [4 tg][9][64][4]
    static_assert(RF <= GF + XF, "exchange fits the staging pool");
    static_assert(HN <= NTB, "one halo pixel per thread");
    __shared__ __attribute__((aligned(16))) float pool[GF + XF];
    float* const Gt = pool;
    unsigned short* const Xt = reinterpret_cast<unsigned short*>(pool + GF);
    __shared__ BnBwdLds coef[SNNFLOW_MAX_WGRAD_STEPS][C];

    const cwgrad_ptr ap = (cwgrad_ptr)__builtin_amdgcn_kernarg_segment_ptr();
    const int tid = threadIdx.x, lane = tid & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nt = wv & 1, mt = (wv >> 1) & 1, rg = wv >> 2;
    const int nsrc = ap->rec ? 2 : 1;
    const int b = blockIdx.x, src = nsrc == 2 ? (b >> 3) & 1 : 0;
    const int bt = nsrc == 2 ? (b & 7) + 8 * (b >> 4) : b;  // tile block index (block_tile's XCD order)
    const int H = ap->H, W = ap->W, nsteps = ap->nsteps;
    const int nbt = ap->B * tiles_per_image(H, W);
    if (bt >= nbt) return;  // padding block (recurrent grid: 2 x the tile count rounded up to 8)
    const Tile tl = block_tile(H, W, Grid{bt, nbt});
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

    for (int e = tid; e < nsteps * C; e += NTB) {
        const int t = e / C, c = e - t * C;
        const float* st = ap->steps[t].stats;
        const float* bc = ap->steps[t].bnc;
        BnBwdLds k = {0.f, 1.f, 0.f, 0.f, 1.f};
        if (st) {
            k.mean = st[c];
            k.inv = st[C + c];
            k.gm = bc[c];
            k.k = bc[C + c];
            k.w = ap->bn_weight[c];
        }
        coef[t][c] = k;
    }

    // the halo pixel of this thread (tid < HN)
    const int hr = tid / HWD, hc = tid - hr * HWD;
    const int hh = tl.h0 + hr - 1, hw = tl.w0 + hc - 1;
    const bool hok = tid < HN && in_image(hh, hw, H, W);
    const int64_t hpix = hok ? ((int64_t)tl.b * H + hh) * W + hw : 0;
    auto in_bits = [&](int t) { return src == 0 ? ap->steps[t].x_bits : ap->steps[t].s_prev_bits; };

    float4 rg4[O::R], ry4[O::R];
    unsigned xw = 0u;
    // the loads are unconditional (an element outside the image reads element 0; the staging zeroes G
    // there): a conditional load made the compiler wait for each pair before issuing the next
    static_assert(O::E % NTB == 0, "every thread holds O::R elements");
    auto issue = [&](int t) {
        const auto& sp = ap->steps[t];
#pragma unroll
        for (int i = 0; i < O::R; ++i) {
            const int e = tid + i * NTB;
            const int p = e / Q, q = e - p * Q;
            const int ty = p / TW, tx = p - ty * TW;
            const int h = tl.h0 + ty, w = tl.w0 + tx;
            const bool ok = h < H && w < W;
            const int64_t k = ok ? (((int64_t)tl.b * H + h) * W + w) * Q + q : 0;
            rg4[i] = reinterpret_cast<const float4*>(sp.g_cur)[k];
            ry4[i] = reinterpret_cast<const float4*>(sp.y)[k];
        }
        const uint8_t* xb = in_bits(t);
        xw = (xb != nullptr && hok) ? spk_load_bits<C>(xb, hpix) : 0u;
    };

    f32x4 acc[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // this wave's MFMAs of the staged step: rows r = rg, rg + 2, ..., the 9 taps of (nt, mt)
    auto compute = [&]() {
#pragma unroll 1
        for (int r = rg; r < TH; r += 2) {
            bf16x8 ah, am, al;
            {
                const int co = mt * 16 + m;
                const float* srcg = Gt + co * GS + r * TW + 8 * g;
                const float4 u = *reinterpret_cast<const float4*>(srcg), v = *reinterpret_cast<const float4*>(srcg + 4);
                const float a8[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const __bf16 h = (__bf16)a8[j];
                    const float r1 = a8[j] - (float)h;
                    const __bf16 md = (__bf16)r1;
                    ah[j] = h;
                    am[j] = md;
                    al[j] = (__bf16)(r1 - (float)md);
                }
            }
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const unsigned short* T = Xt + (nt * 16 + m) * XS + (r + ky) * 40 + 8 * g;
                const u32x4 u = *reinterpret_cast<const u32x4*>(T);
                const uint2 v = *reinterpret_cast<const uint2*>(T + 8);
                const unsigned int w6[5] = {u.x, u.y, u.z, u.w, v.x};
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    u32x4 bw;
                    if (kx == 0) bw = u32x4{w6[0], w6[1], w6[2], w6[3]};
                    else if (kx == 2) bw = u32x4{w6[1], w6[2], w6[3], w6[4]};
                    else bw = u32x4{__builtin_amdgcn_alignbit(w6[1], w6[0], 16), __builtin_amdgcn_alignbit(w6[2], w6[1], 16),
                                    __builtin_amdgcn_alignbit(w6[3], w6[2], 16), __builtin_amdgcn_alignbit(w6[4], w6[3], 16)};
                    const bf16x8 bb = __builtin_bit_cast(bf16x8, bw);
                    f32x4& o = acc[ky * 3 + kx];
                    o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bb, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bb, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bb, o, 0, 0, 0);
                }
            }
        }
    };

    issue(0);
    __syncthreads();  // coef
    for (int t = 0; t < nsteps; ++t) {
        const auto& sp = ap->steps[t];
        // G^T = BN backward of g_cur (zero outside the image), from the prefetched registers
#pragma unroll
        for (int i = 0; i < O::R; ++i) {
            const int e = tid + i * NTB;
            if (e < O::E) {
                const int p = e / Q, q = e - p * Q;
                const int ty = p / TW, tx = p - ty * TW;
                const bool img = tl.h0 + ty < H && tl.w0 + tx < W;
                const float4 gv = img ? bn_bwd4(rg4[i], ry4[i], &coef[t][4 * q]) : z4;
                float* d = Gt + (4 * q) * GS + p;
                d[0] = gv.x;
                d[GS] = gv.y;
                d[2 * GS] = gv.z;
                d[3 * GS] = gv.w;
            }
        }
        // X^T: the conv input of step t (bit plane: the halo pixel's word -> 32 bf16 0 / 1)
        const uint8_t* xb = in_bits(t);
        const float* xf = src == 0 ? sp.x : sp.s_prev;
        const bool have = xb != nullptr || xf != nullptr;
        if (xb != nullptr) {
            if (tid < HN) {
                unsigned short* d = Xt + hr * 40 + hc;
#pragma unroll
                for (int c = 0; c < C; ++c)
                    d[c * XS] = ((xw >> SNNFLOW_SPK_BIT(C, c)) & 1u) ? (unsigned short)0x3F80 : (unsigned short)0;
            }
        } else if (xf != nullptr) {  // fp32 NHWC plane (s_prev at t = 0), element-wise
            for (int e = tid; e < HN * Q; e += NTB) {
                const int64_t k = halo_idx4<C>(e, tl, H, W);
                const float4 v = k >= 0 ? reinterpret_cast<const float4*>(xf)[k] : z4;
                const int p = e / Q, q = e - p * Q;
                const int r = p / HWD, cc = p - r * HWD;
                unsigned short* d = Xt + (4 * q) * XS + r * 40 + cc;
                d[0] = __builtin_bit_cast(unsigned short, (__bf16)v.x);
                d[XS] = __builtin_bit_cast(unsigned short, (__bf16)v.y);
                d[2 * XS] = __builtin_bit_cast(unsigned short, (__bf16)v.z);
                d[3 * XS] = __builtin_bit_cast(unsigned short, (__bf16)v.w);
            }
        }
        __syncthreads();
        if (t + 1 < nsteps) issue(t + 1);  // step t+1's loads fly during step t's MFMAs
        if (have) compute();
        __syncthreads();  // before the next step overwrites the tiles
    }

    // row group 1 adds into row group 0 through LDS (fixed order)
    const int64_t blk = bt;
    const int accumulate = ap->accumulate;
    float* red = pool;
    const int tg = wv & 3;
    if (rg == 1) {
#pragma unroll
        for (int j = 0; j < 9; ++j) *reinterpret_cast<f32x4*>(red + ((tg * 9 + j) * 64 + lane) * 4) = acc[j];
    }
    __syncthreads();
    if (rg == 0) {
        float* slab = (src == 0 ? ap->slab_ff : ap->slab_rec) + blk * (C * C * 9);
        const int ci = nt * 16 + m;
        slab_rmw_36(slab, mt * 16 + 4 * g, ci, accumulate, [&](int j) {
            return acc[j] + *reinterpret_cast<const f32x4*>(red + ((tg * 9 + j) * 64 + lane) * 4);
        });
    }
}

// Sum of per-block weight-gradient slabs in fp64, fixed order: 64 elements x 16 slab
// groups per 1024-thread block, 4 independent accumulators per thread.
constexpr int SR_E = 64, SR_G = 16;

__global__ __launch_bounds__(SR_E * SR_G) void k_slab_reduce(DescBatch<snnflow_slab_desc> batch, int nblk) {
    __shared__ double part[SR_G][SR_E];
    const snnflow_slab_desc d = batch.pick(blockIdx.y);
    const int le = threadIdx.x % SR_E, g = threadIdx.x / SR_E;
    const int e = blockIdx.x * SR_E + le;
    if (blockIdx.x * SR_E >= d.elems) return;  // uniform per block
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    if (e < d.elems) {
        const float* src = d.slab + e;
        const int64_t st = d.elems;
        int b = g;
        for (; b + 3 * SR_G < nblk; b += 4 * SR_G) {
            s0 += src[(int64_t)b * st];
            s1 += src[(int64_t)(b + SR_G) * st];
            s2 += src[(int64_t)(b + 2 * SR_G) * st];
            s3 += src[(int64_t)(b + 3 * SR_G) * st];
        }
        for (; b < nblk; b += SR_G) s0 += src[(int64_t)b * st];
    }
    part[g][le] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (g == 0 && e < d.elems) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < SR_G; ++k) s += part[k][le];
        d.out[e] = (float)s;
    }
}

// torch.nn.utils.clip_grad_norm_ over the engine's flat gradient buffer in one block:
// total = ||g||_2 (fp64 accumulation, fixed order), coef = min(max_norm / (total + eps), 1),
// g *= coef (train_flow.py:265-266).
constexpr int CLIP_NT = 1024;

__global__ __launch_bounds__(CLIP_NT) void k_clip_grad_norm(float* g, int64_t n, float max_norm, float eps,
                                                          float* total_out) {
    __shared__ double part[CLIP_NT / 64];
    __shared__ float coef_s;
    // 8 guarded loads in flight per thread and round (one block: the vector is small, ~5e3..1e5
    // floats; a serial tail loop waited one memory latency per element)
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 8 * CLIP_NT) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = i + k * CLIP_NT < n ? g[i + k * CLIP_NT] : 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += (double)v[k] * (double)v[k];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < CLIP_NT / 64; ++w) t += part[w];
        const float total = (float)sqrt(t);
        float c = max_norm / (total + eps);
        coef_s = c < 1.0f ? c : 1.0f;
        if (total_out) total_out[0] = total;
    }
    __syncthreads();
    const float c = coef_s;
    for (int64_t j = threadIdx.x; j < n; j += 8 * CLIP_NT) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = j + k * CLIP_NT < n ? g[j + k * CLIP_NT] : 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (j + k * CLIP_NT < n) g[j + k * CLIP_NT] = v[k] * c;
    }
}

// clip_grad_norm_ + Adam (snnflow_clip_adam).  Block b owns elements [b S, (b+1) S), S =
// CLIP_PER * CLIP_NT, one round with every load issued before any math.  One block (n <= S): the norm
// pass and the step increment in the same launch.  Several blocks: k_clip_adam_norm writes per-block
// norm partials and increments the step first; every block of k_clip_adam then sums all partials in
// block order (the same value everywhere, deterministic).  Elements find their parameter tensor by a
// binary search over the LDS copy of the table (offsets ascending, host-checked); Adam as the reference
// (torch _single_tensor_adam: lerp first moment, fp64 bias corrections).
constexpr int CLIP_PER = 8, CLIP_SLICE = CLIP_PER * CLIP_NT;
static_assert(CLIP_SLICE == SNNFLOW_CLIP_ADAM_ONE_BLOCK, "one-block size");

__device__ inline double clip_sq_slice(const float* g, int64_t n, int64_t i0, int64_t i1) {
    double s = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += (int64_t)CLIP_SLICE) {
        float v[CLIP_PER];
#pragma unroll
        for (int k = 0; k < CLIP_PER; ++k) v[k] = i + k * CLIP_NT < i1 ? g[i + k * CLIP_NT] : 0.0f;
#pragma unroll
        for (int k = 0; k < CLIP_PER; ++k) s += (double)v[k] * (double)v[k];
    }
    return s;
}

// block total of a per-thread double (all threads; result valid in thread 0)
__device__ inline double clip_block_sum(double s, double* part) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < CLIP_NT / 64; ++w) t += part[w];
    return t;
}

__global__ __launch_bounds__(CLIP_NT) void k_clip_adam_norm(snnflow_clip_adam_args a) {
    __shared__ double part[CLIP_NT / 64];
    const int64_t i0 = (int64_t)blockIdx.x * CLIP_SLICE, i1 = i0 + CLIP_SLICE < a.n ? i0 + CLIP_SLICE : a.n;
    const double t = clip_block_sum(a.max_norm > 0.0f ? clip_sq_slice(a.grad, a.n, i0, i1) : 0.0, part);
    if (threadIdx.x == 0) {
        a.scratch[blockIdx.x] = t;
        if (blockIdx.x == 0) a.step[0] = a.step[0] + 1.0f;
    }
}

__global__ __launch_bounds__(CLIP_NT) void k_clip_adam(snnflow_clip_adam_args a, int nparts) {
    // Every load of the block (step counter, gradients, parameters, both moments) is issued in one
    // round ahead of the norm reduction: the update needs nothing from the norm but the clip factor,
    // so the kernel waits for one memory latency, not three (norm pass, step counter, update).
    __shared__ double part[CLIP_NT / 64];
    __shared__ float coef_s;
    __shared__ snnflow_adam_tensor tab[SNNFLOW_ADAM_MAX_TENSORS];  // the argument table, for lookups
    if (threadIdx.x < a.ntensors) tab[threadIdx.x] = a.t[threadIdx.x];
    const bool clip = a.max_norm > 0.0f;
    const float st_in = a.step[0];
    __syncthreads();
    const int64_t lo_i = nparts ? (int64_t)blockIdx.x * CLIP_SLICE : 0;
    const int64_t hi_i = lo_i + CLIP_SLICE < a.n ? lo_i + CLIP_SLICE : a.n;  // (one block: n <= CLIP_SLICE)
    float gv[CLIP_PER], pv[CLIP_PER], mv[CLIP_PER], vv[CLIP_PER];
    float *pp[CLIP_PER], *mp[CLIP_PER], *vp[CLIP_PER];
#pragma unroll
    for (int u = 0; u < CLIP_PER; ++u) {  // gradients first: the norm waits only for them
        const int64_t i = lo_i + threadIdx.x + (int64_t)u * CLIP_NT;
        gv[u] = i < hi_i ? a.grad[i] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < CLIP_PER; ++u) {
        const int64_t i = lo_i + threadIdx.x + (int64_t)u * CLIP_NT;
        pp[u] = nullptr;
        if (i >= hi_i) continue;
        int lo = 0, hi = a.ntensors - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (tab[mid].offset <= i) lo = mid;
            else hi = mid - 1;
        }
        const int64_t j = i - tab[lo].offset;
        if (j < 0 || j >= tab[lo].numel) continue;  // a gap between tensors (not written by the engine)
        pp[u] = tab[lo].param + j;
        mp[u] = a.exp_avg + tab[lo].state_offset + j;
        vp[u] = a.exp_avg_sq + tab[lo].state_offset + j;
        pv[u] = *pp[u];
        mv[u] = *mp[u];
        vv[u] = *vp[u];
    }
    double tot = 0.0;
    if (nparts == 0) {  // one block: the norm over all n here (the same squares, the same order)
        double sq = 0.0;
        if (clip) {
#pragma unroll
            for (int u = 0; u < CLIP_PER; ++u) sq += (double)gv[u] * (double)gv[u];
        }
        tot = clip_block_sum(sq, part);
    } else if (threadIdx.x == 0 && clip) {
        for (int j = 0; j < nparts; ++j) tot += a.scratch[j];
    }
    // the step counter: incremented here (one block) or by k_clip_adam_norm (several)
    const float st = nparts == 0 ? st_in + 1.0f : st_in;
    if (threadIdx.x == 0) {
        if (clip) {
            const float total = (float)sqrt(tot);
            const float cc = a.max_norm / (total + a.clip_eps);
            coef_s = cc < 1.0f ? cc : 1.0f;
            if (a.total_out && blockIdx.x == 0) a.total_out[0] = total;
        } else {
            coef_s = 1.0f;
        }
        if (nparts == 0) a.step[0] = st;
    }
    const double step = (double)st;
    const double bc1 = 1.0 - pow(a.beta1, step), bc2 = 1.0 - pow(a.beta2, step);  // (overlaps the barrier wait)
    __syncthreads();
    const float c = coef_s;
    const float neg_step_size = (float)(-(a.lr / bc1));
    const float bc2_sqrt = (float)sqrt(bc2);
    const float w1 = (float)(1.0 - a.beta1), b2 = (float)a.beta2, w2 = (float)(1.0 - a.beta2);
    const float eps = (float)a.eps, wd = (float)a.weight_decay;
#pragma unroll
    for (int u = 0; u < CLIP_PER; ++u) {
        if (!pp[u]) continue;
        float g = gv[u];
        if (clip) {
            g = g * c;
            a.grad[lo_i + threadIdx.x + (int64_t)u * CLIP_NT] = g;  // clip_grad_norm_ scales the gradients in place
        }
        float p = pv[u];
        if (wd != 0.0f) g = g + wd * p;
        const float m = mv[u] + w1 * (g - mv[u]);  // lerp, weight < 0.5
        const float v = vv[u] * b2 + w2 * g * g;
        const float denom = sqrtf(v) / bc2_sqrt + eps;
        p = p + neg_step_size * (m / denom);
        *mp[u] = m;
        *vp[u] = v;
        *pp[u] = p;
    }
}

__global__ void k_lif_export(const float* __restrict__ x, const float* __restrict__ mem, const float* __restrict__ beta,
                             const float* __restrict__ thr, int64_t total, int C, int HW, float* spk, float* mout) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)((i / HW) % C);
        const float m = beta[c] * mem[i] + x[i];
        const bool s = m >= thr[c];
        spk[i] = s ? 1.0f : 0.0f;
        mout[i] = s ? 0.0f : m;
    }
}

// ---------------------------------------------------------------------------
// Wavefront launches (snnflow_fwd_slot / snnflow_bwd_slot): the blocks of one launch are
// split into per-task ranges (each a multiple of 8 blocks, so a task's block -> tile map
// keeps its XCD grouping); every block runs the body of its task's kernel variant on its
// own range (Grid), out of one LDS pool sized for the largest variant.
// ---------------------------------------------------------------------------
constexpr int kSlotTasks = SNNFLOW_MAX_SLOT_TASKS;

enum SlotKind : int {
    SK_HEAD1, SK_HEAD2, SK_HEAD4, SK_HEAD5,  // conv of a cin-channel input (no LIF)
    SK_PLAIN, SK_PLAIN_REC,                  // conv of a C-channel input (no LIF) [+ rec]
    SK_LIF, SK_LIF_REC,                      // LIF(l-1) on the halo + conv(l) [+ rec]
    SK_TOP, SK_TOP_PRED,                     // LIF of the last layer [+ pred]
    SK_LIF_P, SK_LIF_REC_P                   // C = 8 forward SK_LIF / SK_LIF_REC as a tile pipeline (fwd_lif8_pipe)
};

struct FwdSlotParams {
    snnflow_conv_fwd_args conv[kSlotTasks];
    snnflow_lif_fwd_args lif;
    int kind[kSlotTasks], blk0[kSlotTasks], nblk[kSlotTasks];
    int ntask;
};
struct BwdSlotParams {
    snnflow_layer_bwd_args layer[kSlotTasks];
    snnflow_lif_bwd_args lif;
    int kind[kSlotTasks], blk0[kSlotTasks], nblk[kSlotTasks];
    int ntask;
};

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// Task kinds compiled into the slot kernels: every kind at C = 8; at C = 16 / 32 only those of the
// LIFFireNet family (2- or 4-bin head, LIF-fed layers, top LIF): the plain C-channel convs would set
// the pool to ~100 KB and the registers to ~146, i.e. one block per CU for every task.
template <int C>
constexpr bool kSlotAllKinds = C == 8;

constexpr int kFragC8 = 3 * 3 * 256;  // bf16 entries per conv of the compact C = 8 fragments (FragC8)
// LDS of the pipeline (bytes): raw y / m halos (680 16-B DMA slots each), the bf16 spike
// tiles (layer l-1, and s_prev for the recurrent conv), the compact fragments.
constexpr int kPipeRaw = 2 * HN * 16, kPipeSpk = HN * 8 * 2, kPipeFrag = kFragC8 * 2;
template <bool REC>
struct PipeFwdLds {
    static constexpr int RAWY = 0, RAWM = kPipeRaw, SPK = 2 * kPipeRaw, RSPK = SPK + kPipeSpk;
    static constexpr int FF = RSPK + (REC ? kPipeSpk : 0), FR = FF + kPipeFrag;
    static constexpr int BYTES = FR + (REC ? kPipeFrag : 0);
    static constexpr int FLOATS = BYTES / 4;
};

template <int C>
struct SlotLds {
    static constexpr int FWD_ALL = cmax(cmax(ConvFwdLds<1, C, false, false, 2>::FLOATS, ConvFwdLds<5, C, false, false, 2>::FLOATS),
                                        cmax(ConvFwdLds<C, C, false, false, 2>::FLOATS, ConvFwdLds<C, C, false, true, 2>::FLOATS));
    static constexpr int FWD_P = C == 8 ? PipeFwdLds<true>::FLOATS : 0;  // the tile pipeline (C = 8)
    static constexpr int FWD = cmax(cmax(cmax(kSlotAllKinds<C> ? FWD_ALL : 0, kLifQFwdLds<C>), FWD_P),
                                    cmax(cmax(ConvFwdLds<2, C, false, false, 2>::FLOATS, ConvFwdLds<4, C, false, false, 2>::FLOATS),
                                         cmax(ConvFwdLds<C, C, true, false, 2>::FLOATS, ConvFwdLds<C, C, true, true, 2>::FLOATS)));
    static constexpr bool BFG = C >= 16;  // LIF-fed layers: bf16 six-product input gradients from global fragments
    static constexpr int BWD_ALL = cmax(LayerBwdLds<C, C, false, false, 2>::FLOATS, LayerBwdLds<C, C, false, true, 2>::FLOATS);
    static constexpr int BWD = cmax(cmax(cmax(kSlotAllKinds<C> ? BWD_ALL : 0, kLifQBwdLds<C, true>),
                                         cmax(LayerBwdLds<2, C, false, false, 2>::FLOATS, LayerBwdLds<4, C, false, false, 2>::FLOATS)),
                                    cmax(LayerBwdLds<C, C, true, false, 2, BFG>::FLOATS,
                                         LayerBwdLds<C, C, true, true, 2, BFG>::FLOATS));
};

// A by-value copy of a kernarg-resident struct (dword loads from the constant address
// space: scalar loads; the fields a body never reads are dead and vanish).
template <typename T>
__device__ inline T kernarg_copy(const __attribute__((address_space(4))) T* p) {
    static_assert(sizeof(T) % 4 == 0, "dword-sized struct");
    T r;
    const __attribute__((address_space(4))) int* src = (const __attribute__((address_space(4))) int*)p;
    int* dst = reinterpret_cast<int*>(&r);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) dst[i] = src[i];
    return r;
}

// The copy above loses the address space of the pointers (kernel arguments are global; a struct
// rebuilt from kernarg dwords is generic), and generic pointers compile to flat_* instructions,
// which count on the LDS counter too: every LDS wait of a body then also waited for its
// outstanding HBM loads and stores.  An empty asm hands each pointer back as a global one.
template <typename T>
__device__ inline T* as_global_ptr(T* p) {
    __attribute__((address_space(1))) T* g;
    asm("" : "=s"(g) : "0"(p));
    return (T*)g;
}
#define SNN_G(x) (x) = as_global_ptr(x)

__device__ inline void globalize(snnflow_neuron& n) {
    SNN_G(n.bn_weight); SNN_G(n.bn_bias); SNN_G(n.running_mean); SNN_G(n.running_var);
    SNN_G(n.num_batches_tracked); SNN_G(n.beta); SNN_G(n.threshold);
}
__device__ inline void globalize(snnflow_neuron_grad& n) {
    SNN_G(n.bn_weight); SNN_G(n.bn_bias); SNN_G(n.beta); SNN_G(n.threshold);
}
__device__ inline void globalize(snnflow_conv_fwd_args& a) {
    SNN_G(a.x); SNN_G(a.prev_y); SNN_G(a.prev_mem); SNN_G(a.prev_acc); SNN_G(a.prev_stats);
    globalize(a.prev);
    SNN_G(a.prev_state); SNN_G(a.wt_ff); SNN_G(a.wt_rec); SNN_G(a.wt_ff_t); SNN_G(a.wt_rec_t); SNN_G(a.s_prev);
    SNN_G(a.prev_spk_bits); SNN_G(a.s_prev_bits);
    SNN_G(a.y); SNN_G(a.acc); SNN_G(a.zero0); SNN_G(a.zero1); SNN_G(a.wf_ff); SNN_G(a.wf_rec);
}
__device__ inline void globalize(snnflow_lif_fwd_args& a) {
    SNN_G(a.y); SNN_G(a.mem); SNN_G(a.acc); SNN_G(a.stats);
    globalize(a.n);
    SNN_G(a.state); SNN_G(a.pred_w); SNN_G(a.pred_b); SNN_G(a.flow); SNN_G(a.zero0); SNN_G(a.zero1);
}
__device__ inline void globalize(snnflow_lif_bwd_args& a) {
    SNN_G(a.y); SNN_G(a.mem); SNN_G(a.stats);
    globalize(a.n);
    SNN_G(a.g_out); SNN_G(a.g_state); SNN_G(a.pred_w); SNN_G(a.flow); SNN_G(a.g_flow); SNN_G(a.g_cur);
    SNN_G(a.g_mem); SNN_G(a.acc); SNN_G(a.zero0); SNN_G(a.zero1);
}
__device__ inline void globalize(snnflow_layer_bwd_args& a) {
    SNN_G(a.y); SNN_G(a.stats); SNN_G(a.g_cur); SNN_G(a.acc_in);
    globalize(a.n);
    globalize(a.ng);
    SNN_G(a.g_pred_w); SNN_G(a.g_pred_b); SNN_G(a.bnc_out); SNN_G(a.wt_bwd_ff); SNN_G(a.wt_bwd_rec);
    SNN_G(a.wt_fwd_ff); SNN_G(a.wt_fwd_rec); SNN_G(a.g_x); SNN_G(a.g_state_prev); SNN_G(a.prev_y);
    SNN_G(a.prev_mem); SNN_G(a.prev_stats);
    globalize(a.prev);
    SNN_G(a.prev_g_state); SNN_G(a.prev_g_cur); SNN_G(a.prev_g_mem); SNN_G(a.acc_out); SNN_G(a.zero0);
    SNN_G(a.zero1); SNN_G(a.wd_ff); SNN_G(a.wd_rec); SNN_G(a.wslab_ff); SNN_G(a.wslab_rec); SNN_G(a.s_prev);
    SNN_G(a.x);
}
__device__ inline void globalize(snnflow_eval_fwd_args& a) {
    SNN_G(a.x); SNN_G(a.s_in); SNN_G(a.mem_prev); SNN_G(a.s_prev); SNN_G(a.wt_ff); SNN_G(a.wt_rec);
    SNN_G(a.wt_ff_t); SNN_G(a.wt_rec_t);
    globalize(a.n);
    SNN_G(a.state); SNN_G(a.pred_w); SNN_G(a.pred_b); SNN_G(a.flow);
}
#undef SNN_G

// A task's argument struct from the kernarg segment, pointers global.
template <typename T>
__device__ inline T task_args(const __attribute__((address_space(4))) T* p) {
    T r = kernarg_copy(p);
    globalize(r);
    return r;
}

// Task of this block (block ranges ascending; ntask <= kSlotTasks) and its Grid.
template <typename P>
__device__ inline int slot_task(const __attribute__((address_space(4))) P* pp, Grid& g) {
    const int bid = blockIdx.x, nt = pp->ntask;
    int k = 0;
#pragma unroll
    for (int i = 1; i < kSlotTasks; ++i)
        if (i < nt && bid >= pp->blk0[i]) k = i;
    g.bid = bid - pp->blk0[k];
    g.nb = pp->nblk[k];
    return k;
}

// ---------------------------------------------------------------------------
// C = 8 LIF-fed forward layer-steps as a tile pipeline (slot kinds SK_LIF_P / SK_LIF_REC_P).
//
// The one-tile-per-block bodies run in lockstep rounds: every block of a round issues its halo
// loads at once (HBM busy), then computes while HBM idles, and the next round starts when the
// whole round is done (phase trace, profiles/r03/ktrace_slot_r3_fused.json: prologue 3.2 of
// 6.1 us per block).  Here a block owns tiles v = bid, bid + nb, ... of its layer-step and
// overlaps tile i's math with tile i+1's loads:
//   * the previous layer's pre-BN current y and membrane m of the next tile's halo go from
//     global memory straight into LDS by LDS-DMA (buffer_load_dwordx4 ... lds; pixels outside
//     the image read an offset past the buffer's range: zeros) -- no registers held in flight;
//   * the per-block prologue (BatchNorm statistics from the batch-sum shards, running-stat
//     update, weight fragments split into bf16 hi / mid / lo) runs once per block, not per tile;
//   * the conv runs with the operands swapped (A = weights, B = spikes): the accumulator rows
//     are output channels, so a lane holds four consecutive channels of one pixel, and one
//     v_permlane32_swap per register packs the wave's two 16-pixel M-tiles into 64 lanes -- the
//     pre-BN current leaves as one 16-B store per lane (no LDS staging, no barrier) and the
//     batch sums stay in registers over the block's tiles (one set of fp64 atomics per block).
// Per tile: wait(DMA) + barrier -> LIF of layer l-1 over the halo from LDS (state stores,
// spikes as a bf16 tile) -> barrier -> DMA of the next tile -> MFMA -> store.  Two barriers per
// tile.  Same arithmetic as conv_fwd_body<8, 8, true, REC, 2> (the conv in another summation
// order inside the matrix core only where the hardware's k-order differs).
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ inline void vm_wait() {  // s_waitcnt vmcnt(N), the other counters untouched
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// A value the compiler cannot treat as loop-invariant (forces per-iteration recomputation of what
// derives from it instead of holding it in registers across the loop).
__device__ inline int opaque_int(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// Compact C = 8 weight fragments: [chunk 0..2][part hi/mid/lo][lane group g][co 0..7][8 bf16],
// the A operand of the swapped conv (lane (co, g) feeds W[tap 4 chunk + g][co][0..7]); rows
// co 8..15 of the matrix core read rows 0..7 again (their outputs are never used).
struct FragC8 {
    float r[2];
    __device__ inline void load(const float* __restrict__ wB) {  // wB [tap][co][ci]
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = (int)threadIdx.x + i * 2 * NT;
            const int j = e & 7, co = (e >> 3) & 7, g = (e >> 6) & 3, ch = e >> 8, tap = 4 * ch + g;
            r[i] = (e < 768 && tap < 9) ? wB[(tap * 8 + co) * 8 + j] : 0.0f;
        }
    }
    __device__ inline void store(__bf16* f) const {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = (int)threadIdx.x + i * 2 * NT;
            if (e < 768) {
                const float w = r[i];
                const __bf16 h = (__bf16)w;
                const float r1 = w - (float)h;
                const __bf16 md = (__bf16)r1;
                __bf16* d = f + (e >> 8) * 3 * 256 + (e & 255);
                d[0] = h;
                d[256] = md;
                d[512] = (__bf16)(r1 - (float)md);
            }
        }
    }
};

// Tiles per block of a pipelined task (host: snnflow_set_pipe); blocks are a multiple of 8 so a
// block's tiles v = bid + k nb stay in its XCD group of block_tile.
__host__ __device__ inline int pipe_tiles(const Grid& g, int ntiles) {
    return g.bid < ntiles ? (ntiles - 1 - g.bid) / g.nb + 1 : 0;
}

// Per-block scheduling state in LDS (the recurrent input's two alternating exactness flags)
__device__ inline int* pipe_slot() {
    __shared__ int slot[4];
    return slot;
}

template <bool REC>
__device__ void fwd_lif8_pipe(const snnflow_conv_fwd_args& a, const Grid g, float* pool) {
    constexpr int C = 8, NTB = 2 * NT, R = Halo4<C, NTB>::R;
    using L = PipeFwdLds<REC>;
    char* const lds = reinterpret_cast<char*>(pool);
    __shared__ LifCoef coef[C];
    __shared__ double sums[2 * C];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = a.H, W = a.W, ntiles = a.B * tiles_per_image(H, W);
    int* const slot = pipe_slot();
    int v_cur = g.bid < ntiles ? g.bid : -1;  // tiles v = bid, bid + nb, ...
    if (v_cur < 0) return;
    const bool lead = g.bid == 0;
    const bool has_mem = a.prev_mem != nullptr;
    const bool has_rec = REC && a.s_prev != nullptr;
    TRACE_AT(true, REC ? 1 : 0, 0);

    // ---- prologue (once per block): batch-sum shards, neuron parameters, fragments, first tile
    AccGather<2 * C> gat;
    if (a.prev.bn_train) acc_gather_load<2 * C>(a.prev_acc, 2 * C, gat);
    const NeuronRegs nr = load_neuron(a.prev, C, lead);
    FragC8 fz_ff, fz_rec;
    fz_ff.load(a.wt_ff_t);
    if (has_rec) fz_rec.load(a.wt_rec_t);

    const uint32_t nbytes = (uint32_t)a.B * H * W * C * 4;  // < 2^31 (host check)
    const __amdgpu_buffer_rsrc_t rs_y = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.prev_y), (short)0, (int)nbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_m =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(has_mem ? a.prev_mem : a.prev_y), (short)0, (int)nbytes, 0x00020000);
    // the raw halo of tile t: 11 wave-loads of 64 x 16 B per tensor, wave w issues loads w, w + 8, w + 16
    auto issue = [&](const Tile& t, int lane) {
        const int base = ((t.b * H + t.h0 - 1) * W + (t.w0 - 1)) * (C * 4);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int k = wv + 8 * j;
            if (k >= 22) break;
            const bool mem = k >= 11;
            if (mem && !has_mem) continue;
            const int kk = mem ? k - 11 : k, ee = kk * 64 + lane, p = ee >> 1, r = p / HWD, cc = p - r * HWD;
            const bool ok = in_image(t.h0 + r - 1, t.w0 + cc - 1, H, W);
            const uint32_t off = ok ? (uint32_t)(base + (r * W + cc) * (C * 4) + (ee & 1) * 16) : 0x80000000u;
            if (ee < 2 * HN)  // the last wave-load is partial: inactive lanes write no LDS
                __builtin_amdgcn_raw_ptr_buffer_load_lds(mem ? rs_m : rs_y, (lds_void*)(lds + (mem ? L::RAWM : L::RAWY) + kk * 1024),
                                                         16, off, 0, 0, 0);
        }
    };
    float4 rs[R];  // s_prev halo of the next tile (registers, issued one tile ahead)
    auto load_sprev = [&](const Tile& t, int tid) {  // halo_load's element order, 32-bit offsets from the halo origin
        const float4* base = reinterpret_cast<const float4*>(a.s_prev) + (((int64_t)t.b * H + (t.h0 - 1)) * W + (t.w0 - 1)) * 2;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = tid + i * NTB, p = e >> 1, r = p / HWD, cc = p - r * HWD;
            const bool ok = e < 2 * HN && in_image(t.h0 + r - 1, t.w0 + cc - 1, H, W);
            rs[i] = ok ? base[(r * W + cc) * 2 + (e & 1)] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    Tile tl = block_tile(H, W, Grid{v_cur, ntiles});
    issue(tl, lane);
    if (has_rec) load_sprev(tl, tid);
    if (a.prev.bn_train) acc_gather_reduce<2 * C>(gat, sums);
    TRACE_AT(true, REC ? 1 : 0, 1);
    lif_prologue(a.prev, nr, sums, C, (double)a.B * H * W, a.prev_stats, coef, nullptr, lead);
    TRACE_AT(true, REC ? 1 : 0, 2);
    fz_ff.store(reinterpret_cast<__bf16*>(lds + L::FF));
    if (has_rec) fz_rec.store(reinterpret_cast<__bf16*>(lds + L::FR));
    zero_consumed(a.zero0, a.zero1, a.zero_n, g);
    if (tid == 0) slot[2] = 0;  // the s_prev exactness flag of tile 0

    const bool zr = a.prev.zero_reset != 0, spk_skip = a.state_spk_skip != 0;
    const int64_t plane4 = (int64_t)a.B * H * W * 2;
    float4* st4 = reinterpret_cast<float4*>(a.prev_state);
    float bs[4] = {0.f, 0.f, 0.f, 0.f}, bq[4] = {0.f, 0.f, 0.f, 0.f};  // this lane's batch sums
    const __bf16* spk = reinterpret_cast<const __bf16*>(lds + L::SPK);
    const __bf16* rspk = reinterpret_cast<const __bf16*>(lds + L::RSPK);
    TRACE_AT(true, REC ? 1 : 0, 3);

    for ([[maybe_unused]] int k = 0; v_cur >= 0; ++k) {
        vm_wait<0>();     // this wave's DMA and s_prev loads of tile k (and its stores of tile k-1)
        __syncthreads();  // every wave's DMA landed; every wave is done with the spike tiles of k-1
        TRACE_AT(k < 2, REC ? 1 : 0, 4 + 3 * k);
        // the lane's tile-independent index math (halo element, DMA slot, LDS addresses) is redone per
        // tile from an opaque copy of the thread index: hoisted out of the loop it held ~30 registers
        const int tid = opaque_int(threadIdx.x), lane = tid & 63, jj = lane & 15, gg = lane >> 4, qt = tid & 1;
        const LifCoef kc[4] = {coef[4 * qt], coef[4 * qt + 1], coef[4 * qt + 2], coef[4 * qt + 3]};
        // LIF of layer l-1 over the halo (element e = pixel * 2 + channel quad, e = tid + i NTB)
        bool ok = true;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = tid + i * NTB;
            if (e < 2 * HN) {
                const int p = e >> 1, r = p / HWD, cc = p - r * HWD;
                const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
                const float4 yv = *reinterpret_cast<const float4*>(lds + L::RAWY + e * 16);
                const float4 mv = has_mem ? *reinterpret_cast<const float4*>(lds + L::RAWM + e * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
                float4 sv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (in_image(h, w, H, W)) {
                    const Lif4 o = zr ? lif_step4(yv, mv, kc, true) : lif_step4(yv, mv, kc, false);
                    sv = o.s;
                    if (r >= 1 && r <= TH && cc >= 1 && cc <= TW) {
                        const int64_t q = (((int64_t)tl.b * H + h) * W + w) * 2 + qt;
                        st_state4(st4, q, o.mout);
                        if (!spk_skip) st_state4(st4, plane4 + q, o.s);
                    }
                }
                typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                *reinterpret_cast<bf16x4*>(const_cast<__bf16*>(spk) + p * 8 + 4 * qt) =
                    bf16x4{(__bf16)sv.x, (__bf16)sv.y, (__bf16)sv.z, (__bf16)sv.w};
                if (has_rec) {
                    const float4 s = rs[i];
                    ok = ok && exact_bf16(s.x) && exact_bf16(s.y) && exact_bf16(s.z) && exact_bf16(s.w);
                    *reinterpret_cast<bf16x4*>(const_cast<__bf16*>(rspk) + p * 8 + 4 * qt) =
                        bf16x4{(__bf16)s.x, (__bf16)s.y, (__bf16)s.z, (__bf16)s.w};
                }
            }
        }
        // raw halos free, spike tiles complete (and: is s_prev exact in bf16 everywhere?  A wave with an
        // inexact value sets this tile's LDS flag -- two flags alternate over the tiles, the other one
        // is cleared here for the next tile -- instead of __syncthreads_and's three barriers)
        int* const bad = slot + 2;  // pipe_slot()[2..3]
        if (has_rec && __builtin_amdgcn_ballot_w64(!ok) != 0 && lane == 0) bad[k & 1] = 1;
        if (threadIdx.x == 0) bad[(k + 1) & 1] = 0;
        __syncthreads();
        const bool rec_bf = has_rec && bad[k & 1] == 0;
        TRACE_AT(k < 2, REC ? 1 : 0, 5 + 3 * k);
        const int v_nxt = v_cur + g.nb < ntiles ? v_cur + g.nb : -1;
        const Tile cur = tl;
        if (v_nxt >= 0) {
            tl = block_tile(H, W, Grid{v_nxt, ntiles});
            issue(tl, lane);
            if (has_rec) load_sprev(tl, tid);
        }

        // conv(s) of this wave's tile row: A = fragments (rows co), B = spikes (columns: pixels)
        const bf16x8* fff = reinterpret_cast<const bf16x8*>(lds + L::FF) + gg * 8 + (jj & 7);
        const bf16x8* ffr = reinterpret_cast<const bf16x8*>(lds + L::FR) + gg * 8 + (jj & 7);
        f32x4 af[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, ar[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const int tap = 4 * ch + gg, ky = tap / 3, kx = tap - 3 * ky;
            const bf16x8 fh = fff[ch * 96], fm = fff[ch * 96 + 32], fl = fff[ch * 96 + 64];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const int off = ((wv + ky) * HWD + mt * 16 + jj + kx) * 8;
                bf16x8 b = {};
                if (tap < 9) b = *reinterpret_cast<const bf16x8*>(spk + off);
                af[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl, b, af[mt], 0, 0, 0);
                af[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm, b, af[mt], 0, 0, 0);
                af[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh, b, af[mt], 0, 0, 0);
            }
            if (rec_bf) {
                const bf16x8 rh = ffr[ch * 96], rm = ffr[ch * 96 + 32], rl = ffr[ch * 96 + 64];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    const int off = ((wv + ky) * HWD + mt * 16 + jj + kx) * 8;
                    bf16x8 b = {};
                    if (tap < 9) b = *reinterpret_cast<const bf16x8*>(rspk + off);
                    ar[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rl, b, ar[mt], 0, 0, 0);
                    ar[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rm, b, ar[mt], 0, 0, 0);
                    ar[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rh, b, ar[mt], 0, 0, 0);
                }
            }
        }
        // lane -> (M-tile lane >> 5, pixel column jj, channel quad (lane >> 4) & 1) after the swap
        f32x4 yv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float y0 = rec_bf ? af[0][r] + ar[0][r] : af[0][r];  // ff + rec (:540)
            const float y1 = rec_bf ? af[1][r] + ar[1][r] : af[1][r];
            const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, y0), __builtin_bit_cast(unsigned, y1),
                                                             false, false);
            yv[r] = __builtin_bit_cast(float, sw[0]);
        }
        const int qd = (lane >> 4) & 1, h = cur.h0 + wv, w = cur.w0 + (lane >> 5) * 16 + jj;
        const bool in = h < H && w < W;
        if (has_rec && !rec_bf && in) {  // s_prev not binary: the recurrent conv on the vector ALU (exact f32)
            const float* wr = a.wt_rec;  // [tap][ci][co]
#pragma unroll 1
            for (int tp = 0; tp < 9; ++tp) {
                const int hh = h + tp / 3 - 1, ww = w + tp % 3 - 1;
                if (!in_image(hh, ww, H, W)) continue;
                const float* sp = a.s_prev + (((int64_t)cur.b * H + hh) * W + ww) * C;
                for (int ci = 0; ci < C; ++ci) {
                    const float s = sp[ci];
#pragma unroll
                    for (int r = 0; r < 4; ++r) yv[r] = fmaf(wr[(tp * C + ci) * C + 4 * qd + r], s, yv[r]);
                }
            }
        }
        if (in) {
            *reinterpret_cast<float4*>(a.y + (((int64_t)cur.b * H + h) * W + w) * C + 4 * qd) =
                make_float4(yv[0], yv[1], yv[2], yv[3]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                bs[r] += yv[r];
                bq[r] += yv[r] * yv[r];
            }
        }
        TRACE_AT(k < 2, REC ? 1 : 0, 6 + 3 * k);
        v_cur = v_nxt;
    }

    // ---- batch sums of the block's tiles: 16-lane rows by DPP, rows and waves through LDS, fp64 atomics
    if (a.acc) {
        float v[8] = {bs[0], bs[1], bs[2], bs[3], bq[0], bq[1], bq[2], bq[3]};
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += dppf<0xB1>(v[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += dppf<0x4E>(v[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += dppf<0x141>(v[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += dppf<0x140>(v[j]);
        float(*red)[4][8] = reinterpret_cast<float(*)[4][8]>(sum_scratch());  // [wave][16-lane row][8 sums]
        if ((lane & 15) == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) red[wv][lane >> 4][j] = v[j];
        }
        __syncthreads();
        if (tid < 2 * C) {  // sum (tid < 8) or sum of squares of channel c
            const int c = tid & 7, sq = tid >> 3, qd = c >> 2, j = sq * 4 + (c & 3);
            double s = 0.0;
#pragma unroll
            for (int w = 0; w < 8; ++w) s += (double)red[w][qd][j] + (double)red[w][qd + 2][j];
            atomicAdd(acc_shard(a.acc, 2 * C, g.bid) + sq * C + c, s);
        }
    }
}

template <int C>
__global__ __launch_bounds__(NT * 2, C == 8 ? 6 : 1) void k_fwd_slot(FwdSlotParams) {
    typedef const __attribute__((address_space(4))) FwdSlotParams* cptr;
    const cptr pp = (cptr)__builtin_amdgcn_kernarg_segment_ptr();
    Grid g;
    const int k = slot_task(pp, g);
    if (g.bid >= g.nb) return;  // padding block of a range
    __shared__ __attribute__((aligned(16))) float pool[SlotLds<C>::FWD];
    switch (pp->kind[k]) {
#define FWD_CONV(ALL, KIND, ...)                              \
    case KIND: {                                              \
        if constexpr (ALL || kSlotAllKinds<C>) {              \
            const snnflow_conv_fwd_args a = task_args(&pp->conv[k]);         \
            conv_fwd_body<__VA_ARGS__>(a, g, pool);           \
        }                                                     \
        break;                                                \
    }
        FWD_CONV(false, SK_HEAD1, 1, C, false, false, 2)
        FWD_CONV(true, SK_HEAD2, 2, C, false, false, 2)
        FWD_CONV(true, SK_HEAD4, 4, C, false, false, 2)
        FWD_CONV(false, SK_HEAD5, 5, C, false, false, 2)
        FWD_CONV(false, SK_PLAIN, C, C, false, false, 2)
        FWD_CONV(false, SK_PLAIN_REC, C, C, false, true, 2)
        FWD_CONV(true, SK_LIF, C, C, true, false, 2)
        FWD_CONV(true, SK_LIF_REC, C, C, true, true, 2)
#undef FWD_CONV
        case SK_LIF_P:
        case SK_LIF_REC_P: {
            if constexpr (C == 8) {
                {
                    const snnflow_conv_fwd_args a = task_args(&pp->conv[k]);
                    if (pp->kind[k] == SK_LIF_REC_P) fwd_lif8_pipe<true>(a, g, pool);
                    else fwd_lif8_pipe<false>(a, g, pool);
                }
            }
            break;
        }
        case SK_TOP: {  // (LIFFireNet's top layer always carries the prediction: C = 8 only)
            if constexpr (kSlotAllKinds<C>) {
                const snnflow_lif_fwd_args a = task_args(&pp->lif);
                lif_fwd_body<C, false, NT * 2>(a, g);
            }
            break;
        }
        case SK_TOP_PRED: {
            const snnflow_lif_fwd_args a = task_args(&pp->lif);
            if constexpr (C >= 16) lif_fwd_q_body<C, true, NT * 2>(a, g, pool);
            else lif_fwd_body<C, true, NT * 2>(a, g);
            break;
        }
        default: break;
    }
}

// ---------------------------------------------------------------------------
// Evaluation forward (snnflow_eval_slot): conv + BatchNorm (running statistics) + LIF of one layer
// in one task, the prediction fused into the last layer's.  C = 8 LIF-fed layers as a tile pipeline
// organised like fwd_lif8_pipe (2 tiles per block, the next tile's spike halo by LDS-DMA while this
// tile's convs run, swapped-operand convs packed by v_permlane32_swap); the head (event-tensor input,
// real-valued: vector-ALU conv in conv_fwd_body's order) one tile per block.
// ---------------------------------------------------------------------------
constexpr int kEvalTasks = SNNFLOW_EVAL_MAX_TASKS;
enum EvalKind : int { EK_HEAD2, EK_HEAD4, EK_FF, EK_REC };

struct EvalSlotParams {
    snnflow_eval_fwd_args t[kEvalTasks];
    int kind[kEvalTasks], blk0[kEvalTasks], nblk[kEvalTasks];
    int ntask;
};

template <bool REC>
struct EvalLds {  // bytes: raw fp32 spike halo (DMA), bf16 spike tiles, compact fragments
    static constexpr int RAW = 0, SPK = kPipeRaw, RSPK = SPK + kPipeSpk;
    static constexpr int FF = RSPK + (REC ? kPipeSpk : 0), FR = FF + kPipeFrag;
    static constexpr int BYTES = FR + (REC ? kPipeFrag : 0);
    static constexpr int FLOATS = BYTES / 4;
};
constexpr int kEvalLdsFloats = cmax(EvalLds<true>::FLOATS, ConvFwdLds<4, 8, false, false, 2>::FLOATS);

// LIF of 4 channels of one pixel from the pre-BN current (layer's own coefficients) and the
// incoming membrane; writes the state (membrane, spike planes) and returns the spikes.
__device__ inline float4 eval_lif_store(const float4& y, const float4& m, const LifCoef* kc, bool zr, float4* st4,
                                        int64_t q, int64_t plane4) {
    const Lif4 o = zr ? lif_step4(y, m, kc, true) : lif_step4(y, m, kc, false);
    st_state4(st4, q, o.mout);
    st_state4(st4, plane4 + q, o.s);
    return o.s;
}

// Head task: conv of the cin-channel event tensor (conv_fwd_body<CIN, 8, false, false, 2>'s staging
// and per-pixel summation order) -> BN + LIF -> state.  One tile per block.
template <int CIN>
__device__ void eval_head_body(const snnflow_eval_fwd_args& a, const Grid g, float* lds) {
    constexpr int C = 8, NTB = 2 * NT, CO = 4;
    __shared__ LifCoef coef[C];
    const int tid = threadIdx.x, pt = tid % NT, ty = pt / TW, tx = pt - ty * TW;
    const int part = thread_part(), co0 = part * CO;
    const int H = a.H, W = a.W;
    const Tile tl = block_tile(H, W, g);
    const NeuronRegs nr = load_neuron(a.n, C, false);
    const int h = tl.h0 + ty, w = tl.w0 + tx;
    const bool in = h < H && w < W;
    const int64_t q = (((int64_t)tl.b * H + (in ? h : 0)) * W + (in ? w : 0)) * 2 + part;
    const float4 mv = (a.mem_prev && in) ? reinterpret_cast<const float4*>(a.mem_prev)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    stage_strided<CIN, NTB>(a.x, a.xs_b, a.xs_c, a.xs_h, a.xs_w, tl, H, W, lds);
    lif_prologue(a.n, nr, nullptr, C, (double)a.B * H * W, nullptr, coef, nullptr, false);
    __syncthreads();
    float y[CO] = {0.f, 0.f, 0.f, 0.f};
    conv_acc<CIN, C, CO>(lds, a.wt_ff, ty, tx, co0, y);
    if (in)
        eval_lif_store(make_float4(y[0], y[1], y[2], y[3]), mv, coef + co0, a.n.zero_reset != 0,
                       reinterpret_cast<float4*>(a.state), q, (int64_t)a.B * H * W * 2);
}

template <bool REC>
__device__ void eval8_pipe(const snnflow_eval_fwd_args& a, const Grid g, float* pool) {
    constexpr int C = 8, NTB = 2 * NT, R = Halo4<C, NTB>::R;
    using L = EvalLds<REC>;
    char* const lds = reinterpret_cast<char*>(pool);
    __shared__ LifCoef coef[C];
    __shared__ int bad[2];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = a.H, W = a.W, ntiles = a.B * tiles_per_image(H, W);
    int v_cur = g.bid < ntiles ? g.bid : -1;
    if (v_cur < 0) return;
    const bool has_mem = a.mem_prev != nullptr;
    const bool has_rec = REC && a.s_prev != nullptr;
    const bool pred = a.flow != nullptr;

    // ---- prologue (once per block): neuron parameters (running statistics), fragments, first tile
    const NeuronRegs nr = load_neuron(a.n, C, false);
    FragC8 fz_ff, fz_rec;
    fz_ff.load(a.wt_ff_t);
    if (has_rec) fz_rec.load(a.wt_rec_t);
    const uint32_t nbytes = (uint32_t)a.B * H * W * C * 4;  // < 2^31 (host check)
    const __amdgpu_buffer_rsrc_t rs_s = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.s_in), (short)0, (int)nbytes, 0x00020000);
    // the raw spike halo of tile t: 11 wave-loads of 64 x 16 B, wave w issues loads w, w + 8
    auto issue = [&](const Tile& t, int lane) {
        const int base = ((t.b * H + t.h0 - 1) * W + (t.w0 - 1)) * (C * 4);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int k = wv + 8 * j;
            if (k >= 11) break;
            const int ee = k * 64 + lane, p = ee >> 1, r = p / HWD, cc = p - r * HWD;
            const bool ok = in_image(t.h0 + r - 1, t.w0 + cc - 1, H, W);
            const uint32_t off = ok ? (uint32_t)(base + (r * W + cc) * (C * 4) + (ee & 1) * 16) : 0x80000000u;
            if (ee < 2 * HN)  // the last wave-load is partial: inactive lanes write no LDS
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_s, (lds_void*)(lds + L::RAW + k * 1024), 16, off, 0, 0, 0);
        }
    };
    float4 rs[R];  // s_prev halo of the next tile (registers, issued one tile ahead)
    auto load_sprev = [&](const Tile& t, int tid) {
        const float4* base = reinterpret_cast<const float4*>(a.s_prev) + (((int64_t)t.b * H + (t.h0 - 1)) * W + (t.w0 - 1)) * 2;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = tid + i * NTB, p = e >> 1, r = p / HWD, cc = p - r * HWD;
            const bool ok = e < 2 * HN && in_image(t.h0 + r - 1, t.w0 + cc - 1, H, W);
            rs[i] = ok ? base[(r * W + cc) * 2 + (e & 1)] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    Tile tl = block_tile(H, W, Grid{v_cur, ntiles});
    issue(tl, lane);
    if (has_rec) load_sprev(tl, tid);
    lif_prologue(a.n, nr, nullptr, C, (double)a.B * H * W, nullptr, coef, nullptr, false);
    fz_ff.store(reinterpret_cast<__bf16*>(lds + L::FF));
    if (has_rec) fz_rec.store(reinterpret_cast<__bf16*>(lds + L::FR));
    if (tid == 0) bad[0] = 0;

    const bool zr = a.n.zero_reset != 0;
    const int64_t plane4 = (int64_t)a.B * H * W * 2;
    float4* st4 = reinterpret_cast<float4*>(a.state);
    const float4* mem4 = reinterpret_cast<const float4*>(a.mem_prev);
    const __bf16* spk = reinterpret_cast<const __bf16*>(lds + L::SPK);
    const __bf16* rspk = reinterpret_cast<const __bf16*>(lds + L::RSPK);
    const int64_t HWp = (int64_t)H * W;

    for (int k = 0; v_cur >= 0; ++k) {
        vm_wait<0>();     // this wave's DMA and s_prev loads of tile k (and its stores of tile k-1)
        __syncthreads();  // every wave's DMA landed; every wave is done with the spike tiles of k-1
        const int tid = opaque_int(threadIdx.x), lane = tid & 63, jj = lane & 15, gg = lane >> 4, qt = tid & 1;
        // the spike halo as a bf16 tile (pixels outside the image: the DMA read zeros); s_prev likewise
        bool ok = true;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = tid + i * NTB;
            if (e < 2 * HN) {
                const int p = e >> 1;
                const float4 sv = *reinterpret_cast<const float4*>(lds + L::RAW + e * 16);
                typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                *reinterpret_cast<bf16x4*>(const_cast<__bf16*>(spk) + p * 8 + 4 * qt) =
                    bf16x4{(__bf16)sv.x, (__bf16)sv.y, (__bf16)sv.z, (__bf16)sv.w};
                if (has_rec) {
                    const float4 s = rs[i];
                    ok = ok && exact_bf16(s.x) && exact_bf16(s.y) && exact_bf16(s.z) && exact_bf16(s.w);
                    *reinterpret_cast<bf16x4*>(const_cast<__bf16*>(rspk) + p * 8 + 4 * qt) =
                        bf16x4{(__bf16)s.x, (__bf16)s.y, (__bf16)s.z, (__bf16)s.w};
                }
            }
        }
        if (has_rec && __builtin_amdgcn_ballot_w64(!ok) != 0 && lane == 0) bad[k & 1] = 1;
        if (threadIdx.x == 0) bad[(k + 1) & 1] = 0;
        __syncthreads();
        const bool rec_bf = has_rec && bad[k & 1] == 0;
        const int v_nxt = v_cur + g.nb < ntiles ? v_cur + g.nb : -1;
        const Tile cur = tl;
        if (v_nxt >= 0) {
            tl = block_tile(H, W, Grid{v_nxt, ntiles});
            issue(tl, lane);
            if (has_rec) load_sprev(tl, tid);
        }
        // this lane's output: row wv, column (lane >> 5) * 16 + jj, channel quad (lane >> 4) & 1
        const int qd = (lane >> 4) & 1, h = cur.h0 + wv, w = cur.w0 + (lane >> 5) * 16 + jj;
        const bool in = h < H && w < W;
        const int64_t pix = ((int64_t)cur.b * H + (in ? h : 0)) * W + (in ? w : 0);
        const float4 mv = (has_mem && in) ? mem4[pix * 2 + qd] : make_float4(0.f, 0.f, 0.f, 0.f);

        const bf16x8* fff = reinterpret_cast<const bf16x8*>(lds + L::FF) + gg * 8 + (jj & 7);
        const bf16x8* ffr = reinterpret_cast<const bf16x8*>(lds + L::FR) + gg * 8 + (jj & 7);
        f32x4 af[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, ar[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const int tap = 4 * ch + gg, ky = tap / 3, kx = tap - 3 * ky;
            const bf16x8 fh = fff[ch * 96], fm = fff[ch * 96 + 32], fl = fff[ch * 96 + 64];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const int off = ((wv + ky) * HWD + mt * 16 + jj + kx) * 8;
                bf16x8 b = {};
                if (tap < 9) b = *reinterpret_cast<const bf16x8*>(spk + off);
                af[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl, b, af[mt], 0, 0, 0);
                af[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm, b, af[mt], 0, 0, 0);
                af[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh, b, af[mt], 0, 0, 0);
            }
            if (rec_bf) {
                const bf16x8 rh = ffr[ch * 96], rm = ffr[ch * 96 + 32], rl = ffr[ch * 96 + 64];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    const int off = ((wv + ky) * HWD + mt * 16 + jj + kx) * 8;
                    bf16x8 b = {};
                    if (tap < 9) b = *reinterpret_cast<const bf16x8*>(rspk + off);
                    ar[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rl, b, ar[mt], 0, 0, 0);
                    ar[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rm, b, ar[mt], 0, 0, 0);
                    ar[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rh, b, ar[mt], 0, 0, 0);
                }
            }
        }
        f32x4 yv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float y0 = rec_bf ? af[0][r] + ar[0][r] : af[0][r];  // ff + rec (:540)
            const float y1 = rec_bf ? af[1][r] + ar[1][r] : af[1][r];
            const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, y0), __builtin_bit_cast(unsigned, y1),
                                                             false, false);
            yv[r] = __builtin_bit_cast(float, sw[0]);
        }
        if (has_rec && !rec_bf && in) {  // s_prev not binary: the recurrent conv on the vector ALU (exact f32)
            const float* wr = a.wt_rec;  // [tap][ci][co]
#pragma unroll 1
            for (int tp = 0; tp < 9; ++tp) {
                const int hh = h + tp / 3 - 1, ww = w + tp % 3 - 1;
                if (!in_image(hh, ww, H, W)) continue;
                const float* sp = a.s_prev + (((int64_t)cur.b * H + hh) * W + ww) * C;
                for (int ci = 0; ci < C; ++ci) {
                    const float s = sp[ci];
#pragma unroll
                    for (int r = 0; r < 4; ++r) yv[r] = fmaf(wr[(tp * C + ci) * C + 4 * qd + r], s, yv[r]);
                }
            }
        }
        // BatchNorm (running statistics) + LIF of this layer; state out
        const LifCoef kc[4] = {coef[4 * qd], coef[4 * qd + 1], coef[4 * qd + 2], coef[4 * qd + 3]};
        const Lif4 o = zr ? lif_step4(make_float4(yv[0], yv[1], yv[2], yv[3]), mv, kc, true)
                          : lif_step4(make_float4(yv[0], yv[1], yv[2], yv[3]), mv, kc, false);
        if (in) {
            st_state4(st4, pix * 2 + qd, o.mout);
            st_state4(st4, plane4 + pix * 2 + qd, o.s);
        }
        if (pred) {  // ConvLayer(C -> 2, 1x1) + tanh: the pixel's other channel quad from lane ^ 16,
                     // summed in channel order as lif_fwd_body does; lane qd writes output qd
            const float p0 = __shfl_xor(o.s.x, 16, 64), p1 = __shfl_xor(o.s.y, 16, 64);
            const float p2 = __shfl_xor(o.s.z, 16, 64), p3 = __shfl_xor(o.s.w, 16, 64);
            const float s8[8] = {qd ? p0 : o.s.x, qd ? p1 : o.s.y, qd ? p2 : o.s.z, qd ? p3 : o.s.w,
                                 qd ? o.s.x : p0, qd ? o.s.y : p1, qd ? o.s.z : p2, qd ? o.s.w : p3};
            if (in) {
                const float* pw = a.pred_w + qd * C;
                float acc = 0.0f;
#pragma unroll
                for (int c = 0; c < C; ++c) acc = fmaf(pw[c], s8[c], acc);
                a.flow[((int64_t)cur.b * 2 + qd) * HWp + (int64_t)h * W + w] = tanhf(acc + a.pred_b[qd]);
            }
        }
        v_cur = v_nxt;
    }
}

__global__ __launch_bounds__(NT * 2, 6) void k_eval_slot(EvalSlotParams) {
    typedef const __attribute__((address_space(4))) EvalSlotParams* cptr;
    const cptr pp = (cptr)__builtin_amdgcn_kernarg_segment_ptr();
    const int bid = blockIdx.x, nt = pp->ntask;
    int k = 0;
#pragma unroll
    for (int i = 1; i < kEvalTasks; ++i)
        if (i < nt && bid >= pp->blk0[i]) k = i;
    Grid g;
    g.bid = bid - pp->blk0[k];
    g.nb = pp->nblk[k];
    if (g.bid >= g.nb) return;  // padding block of a range
    __shared__ __attribute__((aligned(16))) float pool[kEvalLdsFloats];
    const snnflow_eval_fwd_args a = task_args(&pp->t[k]);
    switch (pp->kind[k]) {
        case EK_HEAD2: eval_head_body<2>(a, g, pool); break;
        case EK_HEAD4: eval_head_body<4>(a, g, pool); break;
        case EK_FF: eval8_pipe<false>(a, g, pool); break;
        case EK_REC: eval8_pipe<true>(a, g, pool); break;
        default: break;
    }
}

#ifndef SNNFLOW_BWD_SLOT_WAVES
#define SNNFLOW_BWD_SLOT_WAVES 6  // min waves per SIMD: 3 blocks per CU (measured: 2 per CU is 15 % slower)
#endif
template <int C>
__global__ __launch_bounds__(NT * 2, C == 8 ? SNNFLOW_BWD_SLOT_WAVES : SNNFLOW_L32_WAVES) void k_bwd_slot(BwdSlotParams) {
    // fused weight gradients (C = 8): the input-gradient results are staged in the two weight-fragment
    // regions, which the pool holds for every task kind
    static_assert(C != 8 || SlotLds<C>::BWD >= LayerBwdLds<C, C, true, true, 2>::FLOATS, "fused wgrad staging");
    static_assert(C != 8 || 2 * LayerBwdLds<C, C, true, true, 2>::FR >= NT * Pad<C>::v, "dgrad staging size");
    // fused head weight gradients: input halo and the accumulators' group scratch behind the G tile
    static_assert(SlotLds<C>::BWD >= LayerBwdLds<2, C, false, false, 2>::G + HN * Pad<2>::v &&
                      SlotLds<C>::BWD >= LayerBwdLds<4, C, false, false, 2>::G + HN * Pad<4>::v &&
                      SlotLds<C>::BWD >= WAcc<2, C, 2 * NT, 0>::SCRATCH && SlotLds<C>::BWD >= WAcc<4, C, 2 * NT, 0>::SCRATCH,
                  "fused head weight gradient staging");
    typedef const __attribute__((address_space(4))) BwdSlotParams* cptr;
    const cptr pp = (cptr)__builtin_amdgcn_kernarg_segment_ptr();
    Grid g;
    const int k = slot_task(pp, g);
    if (g.bid >= g.nb) return;
    __shared__ __attribute__((aligned(16))) float pool[SlotLds<C>::BWD];
    switch (pp->kind[k]) {
#define BWD_LAYER(ALL, KIND, ...)                             \
    case KIND: {                                              \
        if constexpr (ALL || kSlotAllKinds<C>) {              \
            const snnflow_layer_bwd_args a = task_args(&pp->layer[k]);       \
            layer_bwd_body<__VA_ARGS__>(a, g, pool);          \
        }                                                     \
        break;                                                \
    }
        BWD_LAYER(true, SK_HEAD2, 2, C, false, false, 2, false, false, true)
        BWD_LAYER(true, SK_HEAD4, 4, C, false, false, 2, false, false, true)
        BWD_LAYER(false, SK_PLAIN, C, C, false, false, 2)
        BWD_LAYER(false, SK_PLAIN_REC, C, C, false, true, 2)
        BWD_LAYER(true, SK_LIF, C, C, true, false, 2, SlotLds<C>::BFG, C == 8)
        BWD_LAYER(true, SK_LIF_REC, C, C, true, true, 2, SlotLds<C>::BFG, C == 8)
#undef BWD_LAYER
        case SK_TOP: {
            if constexpr (kSlotAllKinds<C>) {
                const snnflow_lif_bwd_args a = task_args(&pp->lif);
                lif_bwd_body<C, false, NT * 2>(a, g);
            }
            break;
        }
        case SK_TOP_PRED: {
            const snnflow_lif_bwd_args a = task_args(&pp->lif);
            if constexpr (C >= 16) lif_bwd_q_body<C, true, NT * 2>(a, g, pool);
            else lif_bwd_body<C, true, NT * 2>(a, g);
            break;
        }
        default: break;
    }
}

// ---------------------------------------------------------------------------
// Host dispatch
// ---------------------------------------------------------------------------
bool valid_c(int c) { return c == 4 || c == 8 || c == 16 || c == 32; }

template <int C>
int conv_fwd_c(const snnflow_conv_fwd_args& a, hipStream_t s) {
    constexpr int SP = C == 32 ? SNNFLOW_SP32 : ((C == 8 || C == 16) ? 2 : 1);  // threads per output pixel
    const dim3 grid(snnflow_conv_blocks(a.B, a.H, a.W)), block(NT * SP);
    if (a.lif_in) {
        if (a.cin != C) SNN_FAIL(SNNFLOW_E_CHANNELS, "conv_fwd: lif_in requires cin == c");
        if (a.wt_rec) hipLaunchKernelGGL((k_conv_fwd<C, C, true, true, SP>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_conv_fwd<C, C, true, false, SP>), grid, block, 0, s, a);
    } else if (a.wt_rec) {  // recurrent cell: input channels C, or the narrow event inputs
        if (a.cin == C) hipLaunchKernelGGL((k_conv_fwd<C, C, false, true, SP>), grid, block, 0, s, a);
        else if (a.cin == 1) hipLaunchKernelGGL((k_conv_fwd<1, C, false, true, SP>), grid, block, 0, s, a);
        else if (a.cin == 2) hipLaunchKernelGGL((k_conv_fwd<2, C, false, true, SP>), grid, block, 0, s, a);
        else if (a.cin == 4) hipLaunchKernelGGL((k_conv_fwd<4, C, false, true, SP>), grid, block, 0, s, a);
        else if (a.cin == 5) hipLaunchKernelGGL((k_conv_fwd<5, C, false, true, SP>), grid, block, 0, s, a);
        else SNN_FAIL(SNNFLOW_E_CHANNELS, "conv_fwd: recurrent cell with unsupported cin (1, 2, 4, 5 or c)");
    } else {
        if (a.cin == 1) hipLaunchKernelGGL((k_conv_fwd<1, C, false, false, SP>), grid, block, 0, s, a);
        else if (a.cin == 2) hipLaunchKernelGGL((k_conv_fwd<2, C, false, false, SP>), grid, block, 0, s, a);
        else if (a.cin == 4) hipLaunchKernelGGL((k_conv_fwd<4, C, false, false, SP>), grid, block, 0, s, a);
        else if (a.cin == 5) hipLaunchKernelGGL((k_conv_fwd<5, C, false, false, SP>), grid, block, 0, s, a);
        else if (a.cin == C) hipLaunchKernelGGL((k_conv_fwd<C, C, false, false, SP>), grid, block, 0, s, a);
        else SNN_FAIL(SNNFLOW_E_CHANNELS, "conv_fwd: unsupported cin");
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

// Blocks of a layer_bwd launch: a layer without any per-pixel output (the head when its input
// needs no gradient and it has no recurrent state gradient to produce) only finishes its neuron
// gradients and BN-backward coefficients, which block 0 does: one block.
int layer_bwd_blocks(const snnflow_layer_bwd_args& a) {
    const bool pixels = a.lif_in || (a.g_x && a.wt_bwd_ff) || (a.wt_bwd_rec && a.g_state_prev) || (a.wslab_ff && a.x);
    return pixels ? snnflow_conv_blocks(a.B, a.H, a.W) : 1;
}

template <int C>
int layer_bwd_c(const snnflow_layer_bwd_args& a, hipStream_t s) {
    constexpr int SP = C == 32 ? SNNFLOW_SP32 : ((C == 8 || C == 16) ? 2 : 1);  // threads per pixel (C x C layers; the head keeps 1)
    const dim3 grid(layer_bwd_blocks(a)), block(NT * SP), block1(NT);
    if (a.lif_in) {
        if (a.cin != C) SNN_FAIL(SNNFLOW_E_CHANNELS, "layer_bwd: lif_in requires cin == c");
        // C = 16 / 32 with pre-split fragments of every conv it transposes: bf16 input gradients
        const bool bfg = C >= 16 && a.wd_ff && (!a.wt_bwd_rec || !a.g_state_prev || a.wd_rec);
        if (bfg) {
            if (a.wt_bwd_rec) hipLaunchKernelGGL((k_layer_bwd<C, C, true, true, SP, C >= 16>), grid, block, 0, s, a);
            else hipLaunchKernelGGL((k_layer_bwd<C, C, true, false, SP, C >= 16>), grid, block, 0, s, a);
        } else if (a.wt_bwd_rec) hipLaunchKernelGGL((k_layer_bwd<C, C, true, true, SP>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_layer_bwd<C, C, true, false, SP>), grid, block, 0, s, a);
    } else if (a.wt_bwd_rec) {  // recurrent cell: input channels C, or the narrow event inputs
        if (a.cin == C) hipLaunchKernelGGL((k_layer_bwd<C, C, false, true, SP>), grid, block, 0, s, a);
        else if (a.cin == 1) hipLaunchKernelGGL((k_layer_bwd<1, C, false, true, 1>), grid, block1, 0, s, a);
        else if (a.cin == 2) hipLaunchKernelGGL((k_layer_bwd<2, C, false, true, 1>), grid, block1, 0, s, a);
        else if (a.cin == 4) hipLaunchKernelGGL((k_layer_bwd<4, C, false, true, 1>), grid, block1, 0, s, a);
        else if (a.cin == 5) hipLaunchKernelGGL((k_layer_bwd<5, C, false, true, 1>), grid, block1, 0, s, a);
        else SNN_FAIL(SNNFLOW_E_CHANNELS, "layer_bwd: recurrent cell with unsupported cin (1, 2, 4, 5 or c)");
    } else {
        if (a.cin == 1) hipLaunchKernelGGL((k_layer_bwd<1, C, false, false, 1>), grid, block1, 0, s, a);
        else if (a.cin == 2) hipLaunchKernelGGL((k_layer_bwd<2, C, false, false, 1>), grid, block1, 0, s, a);
        else if (a.cin == 4) hipLaunchKernelGGL((k_layer_bwd<4, C, false, false, 1>), grid, block1, 0, s, a);
        else if (a.cin == 5) hipLaunchKernelGGL((k_layer_bwd<5, C, false, false, 1>), grid, block1, 0, s, a);
        else if (a.cin == C) hipLaunchKernelGGL((k_layer_bwd<C, C, false, false, SP>), grid, block, 0, s, a);
        else SNN_FAIL(SNNFLOW_E_CHANNELS, "layer_bwd: unsupported cin");
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

int elem_grid(int64_t n) {
    int64_t g = (n + NT - 1) / NT;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" {

int snnflow_abi_version(void) { return SNNFLOW_ABI_VERSION; }

#if SNNFLOW_TRACE
int snnflow_trace_copy(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_trace), bytes < sizeof(g_trace) ? bytes : sizeof(g_trace), 0,
                                    hipMemcpyDeviceToHost);
}
#endif
const char* snnflow_last_error(void) { return g_err.c_str(); }

int snnflow_conv_blocks(int B, int H, int W) { return B * tiles_per_image(H, W); }

int snnflow_frag_halfs(int c, int cin) {
    if (cin != c || c <= 0 || c % 8 != 0 || c > 64) return 0;
    return FragGeo(c, c).halfs();
}

int snnflow_prep_weights_batch(const snnflow_prep_desc* d, int n, void* stream) {
    if (!d || n <= 0 || n > SNNFLOW_MAX_BATCH) SNN_FAIL(SNNFLOW_E_ARG, "prep_weights_batch: bad count");
    DescBatch<snnflow_prep_desc> batch = {};
    int maxe = 1;
    for (int i = 0; i < n; ++i) {
        const snnflow_prep_desc& x = d[i];
        if ((x.w && (x.c <= 0 || x.cin <= 0 || !x.wt_fwd || !x.wt_bwd)) || (!x.w && !x.threshold && !x.zero) ||
            (x.threshold && x.thr_n <= 0) || (x.zero && x.zero_n < 0))
            SNN_FAIL(SNNFLOW_E_ARG, "prep_weights_batch: bad descriptor");
        if ((x.frag_fwd || x.frag_bwd) && (!x.w || snnflow_frag_halfs(x.c, x.cin) == 0))
            SNN_FAIL(SNNFLOW_E_ARG, "prep_weights_batch: fragments need cin == c, c % 8 == 0");
        batch.d[i] = x;
        if (x.w && x.c * x.cin * 9 > maxe) maxe = x.c * x.cin * 9;
        if (x.frag_fwd || x.frag_bwd) {
            const int fe = snnflow_frag_halfs(x.c, x.cin) / 3;
            if (fe > maxe) maxe = fe;
        }
        if (x.threshold && x.thr_n > maxe) maxe = x.thr_n;
        if (x.zero) maxe = std::max(maxe, (int)std::min<int64_t>(x.zero_n, 65536));  // grid-stride beyond
    }
    hipLaunchKernelGGL(k_prep_weights, dim3((maxe + 255) / 256, n), dim3(256), 0, (hipStream_t)stream, batch);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_prep_weights(const float* w, int c, int cin, float* wt_fwd, float* wt_bwd, float* threshold,
                         void* stream) {
    if (c <= 0 || cin <= 0 || (w && (!wt_fwd || !wt_bwd)) || (!w && !threshold))
        SNN_FAIL(SNNFLOW_E_ARG, "prep_weights: bad args");
    snnflow_prep_desc d = {w, c, cin, wt_fwd, wt_bwd, threshold, c, nullptr, nullptr, nullptr, 0};
    return snnflow_prep_weights_batch(&d, 1, stream);
}

static int conv_fwd_check(const snnflow_conv_fwd_args* a) {
    if (!a || a->B <= 0 || a->H <= 0 || a->W <= 0 || !a->wt_ff || !a->y)
        SNN_FAIL(SNNFLOW_E_ARG, "conv_fwd: bad args");
    if (a->cin == a->c && a->c % 8 == 0 && (!a->wt_ff_t || (a->wt_rec && !a->wt_rec_t)))
        SNN_FAIL(SNNFLOW_E_ARG, "conv_fwd: cin == c needs the backward-layout weights wt_ff_t / wt_rec_t");
    if (a->lif_in ? (!a->prev_y || !a->prev_state || (a->prev.bn_train && !a->prev_acc)) : !a->x)
        SNN_FAIL(SNNFLOW_E_ARG, "conv_fwd: missing input");
    const bool bits_ok = a->cin == a->c && (a->c == 8 || a->c == 16 || a->c == 32);
    if ((a->prev_spk_bits && !(bits_ok && a->lif_in)) || (a->s_prev_bits && !(bits_ok && a->wt_rec)))
        SNN_FAIL(SNNFLOW_E_ARG, "conv_fwd: spike bit planes need cin == c in {8, 16, 32} (and lif_in / a recurrent conv)");
    return 0;
}

int snnflow_conv_fwd(const snnflow_conv_fwd_args* a, void* stream) {
    if (const int e = conv_fwd_check(a)) return e;
    const hipStream_t s = (hipStream_t)stream;
    switch (a->c) {
        case 4: return conv_fwd_c<4>(*a, s);
        case 8: return conv_fwd_c<8>(*a, s);
        case 16: return conv_fwd_c<16>(*a, s);
        case 32: return conv_fwd_c<32>(*a, s);
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "conv_fwd: c must be 4, 8, 16 or 32");
    }
}

static int lif_fwd_check(const snnflow_lif_fwd_args* a) {
    if (!a || !a->y || !a->state || a->B <= 0 || a->H <= 0 || a->W <= 0 || (a->n.bn_train && !a->acc))
        SNN_FAIL(SNNFLOW_E_ARG, "lif_fwd: bad args");
    if (a->pred_w && (!a->pred_b || !a->flow)) SNN_FAIL(SNNFLOW_E_ARG, "lif_fwd: pred needs bias and flow");
    return 0;
}

int snnflow_lif_fwd(const snnflow_lif_fwd_args* a, void* stream) {
    if (const int e = lif_fwd_check(a)) return e;
    const hipStream_t s = (hipStream_t)stream;
    const int64_t npix = (int64_t)a->B * a->H * a->W;
    // C <= 8: one thread per pixel (measured faster there); C >= 16: quad layout
    const int items = lifq_items(npix, a->c, kLifQFwdBlocks);
    const dim3 grid(a->c >= 16 ? lifq_grid(npix, a->c, items) : elem_grid(npix)), block(NT);
    const bool pred = a->pred_w != nullptr;
    switch (a->c) {
#define LIF_FWD_CASE(CC)                                                                     \
    case CC:                                                                                 \
        if (pred) hipLaunchKernelGGL((k_lif_fwd<CC, true>), grid, block, 0, s, *a);          \
        else hipLaunchKernelGGL((k_lif_fwd<CC, false>), grid, block, 0, s, *a);              \
        break;
#define LIF_FWD_Q_CASE(CC)                                                                   \
    case CC:                                                                                 \
        if (pred) hipLaunchKernelGGL((k_lif_fwd_q<CC, true>), grid, block, 0, s, *a); \
        else hipLaunchKernelGGL((k_lif_fwd_q<CC, false>), grid, block, 0, s, *a);     \
        break;
        LIF_FWD_CASE(4) LIF_FWD_CASE(8) LIF_FWD_Q_CASE(16) LIF_FWD_Q_CASE(32)
#undef LIF_FWD_Q_CASE
#undef LIF_FWD_CASE
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "lif_fwd: c must be 4, 8, 16 or 32");
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

static int lif_bwd_check(const snnflow_lif_bwd_args* a) {
    if (!a || !a->y || !a->stats || !a->g_cur || !a->acc) SNN_FAIL(SNNFLOW_E_ARG, "lif_bwd: bad args");
    if (a->pred_w && !a->flow) SNN_FAIL(SNNFLOW_E_ARG, "lif_bwd: pred needs flow");
    if (a->mem_grad_in && a->pred_w) SNN_FAIL(SNNFLOW_E_ARG, "lif_bwd: mem_grad_in without prediction only");
    return 0;
}

int snnflow_lif_bwd(const snnflow_lif_bwd_args* a, void* stream) {
    if (const int e = lif_bwd_check(a)) return e;
    const bool pred = a->pred_w != nullptr;
    const hipStream_t s = (hipStream_t)stream;
    const int64_t npix = (int64_t)a->B * a->H * a->W;
    const int items = lifq_items(npix, a->c, kLifQBwdBlocks);
    const dim3 grid(a->c >= 16 ? lifq_grid(npix, a->c, items) : elem_grid(npix)), block(NT);
    switch (a->c) {
#define LIF_BWD_CASE(CC)                                                                     \
    case CC:                                                                                 \
        if (pred) hipLaunchKernelGGL((k_lif_bwd<CC, true>), grid, block, 0, s, *a);          \
        else hipLaunchKernelGGL((k_lif_bwd<CC, false>), grid, block, 0, s, *a);              \
        break;
#define LIF_BWD_Q_CASE(CC)                                                                   \
    case CC:                                                                                 \
        if (pred) hipLaunchKernelGGL((k_lif_bwd_q<CC, true>), grid, block, 0, s, *a); \
        else hipLaunchKernelGGL((k_lif_bwd_q<CC, false>), grid, block, 0, s, *a);     \
        break;
        LIF_BWD_CASE(4) LIF_BWD_CASE(8) LIF_BWD_Q_CASE(16) LIF_BWD_Q_CASE(32)
#undef LIF_BWD_Q_CASE
#undef LIF_BWD_CASE
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "lif_bwd: c must be 4, 8, 16 or 32");
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_lif_theta_subtract(const float* g_cur, const float* mem, const float* thr, int64_t npix, int c,
                               float* g_theta, float* scratch, void* stream) {
    if (!g_cur || !mem || !thr || !g_theta || !scratch || npix <= 0)
        SNN_FAIL(SNNFLOW_E_ARG, "lif_theta_subtract: bad args");
    const int64_t n4 = npix * (c / 4);
    int64_t g = (n4 + NT - 1) / NT;
    if (g > SNNFLOW_THETA_BLOCKS) g = SNNFLOW_THETA_BLOCKS;
    const dim3 grid((unsigned)g), block(NT);
    const hipStream_t s = (hipStream_t)stream;
    switch (c) {
        case 4: hipLaunchKernelGGL(k_lif_theta_subtract<4>, grid, block, 0, s, g_cur, mem, thr, npix, scratch); break;
        case 8: hipLaunchKernelGGL(k_lif_theta_subtract<8>, grid, block, 0, s, g_cur, mem, thr, npix, scratch); break;
        case 16: hipLaunchKernelGGL(k_lif_theta_subtract<16>, grid, block, 0, s, g_cur, mem, thr, npix, scratch); break;
        case 32: hipLaunchKernelGGL(k_lif_theta_subtract<32>, grid, block, 0, s, g_cur, mem, thr, npix, scratch); break;
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "lif_theta_subtract: c must be 4, 8, 16 or 32");
    }
    SNN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_lif_theta_reduce, dim3(1), dim3(64), 0, s, scratch, (int)g, c, g_theta);
    SNN_CHECK_LAUNCH();
    return 0;
}

static int layer_bwd_check(const snnflow_layer_bwd_args* a) {
    if (!a || !a->y || !a->stats || !a->g_cur || !a->acc_in) SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: bad args");
    if (!a->ng.bn_weight || !a->ng.bn_bias || !a->ng.beta || !a->ng.threshold)
        SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: missing parameter-gradient buffers");
    if (a->has_pred && (!a->g_pred_w || !a->g_pred_b)) SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: pred gradients");
    if (a->lif_in && (!a->wt_bwd_ff || !a->prev_y || !a->prev_stats || !a->prev_g_cur || !a->acc_out))
        SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: lif_in needs previous-layer buffers");
    if (a->cin == a->c && a->c % 8 == 0 &&
        ((a->wt_bwd_ff && !a->wt_fwd_ff) || (a->wt_bwd_rec && a->g_state_prev && !a->wt_fwd_rec)))
        SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: cin == c needs the forward-layout weights wt_fwd_ff / wt_fwd_rec");
    return 0;
}

int snnflow_layer_bwd(const snnflow_layer_bwd_args* a, void* stream) {
    if (const int e = layer_bwd_check(a)) return e;
    const hipStream_t s = (hipStream_t)stream;
    switch (a->c) {
        case 4: return layer_bwd_c<4>(*a, s);
        case 8: return layer_bwd_c<8>(*a, s);
        case 16: return layer_bwd_c<16>(*a, s);
        case 32: return layer_bwd_c<32>(*a, s);
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "layer_bwd: c must be 4, 8, 16 or 32");
    }
}

// C = 8 only: one layer-step of C = 16 / 32 already fills the chip for a launch (and the
// merged variants would spill registers there).
static bool slot_c(int c) { return c == 8 || c == 16 || c == 32; }

// Block order of a wavefront launch at C = 16 / 32: the blocks are dispatched in index order, so
// the tasks whose blocks live longest (recurrent convs, then the other LIF-fed convs, then heads)
// take the first ranges and the short ones fill the last round (the top task is always last).
// Measured (profiles/r02/ab_slot_order.txt): C = 32 6.50 -> 6.435 ms; at C = 8 the same order is
// slower (fwd slot 20.9 -> 21.8 us), which keeps the layer order.
#ifndef SNNFLOW_SLOT_ORDER
#define SNNFLOW_SLOT_ORDER 1
#endif
static int slot_rank(int kind) {
    switch (kind) {
        case SK_LIF_REC_P: case SK_LIF_P: return 0;
        case SK_LIF_REC: case SK_PLAIN_REC: return 0;
        case SK_LIF: case SK_PLAIN: return 1;
        default: return 2;
    }
}

#ifndef SNNFLOW_SLOT_ORDER8
#define SNNFLOW_SLOT_ORDER8 0  // C = 8: 0 layer order, 1 longest first, 2 shortest first (A/B only)
#endif
extern "C++" template <typename A>
static void slot_sort(A* args, int* kind, int* nblk, int n, bool reverse = false) {
    if (!SNNFLOW_SLOT_ORDER) return;
    const int sg = reverse ? -1 : 1;
    for (int i = 1; i < n; ++i)  // stable insertion sort by rank
        for (int j = i; j > 0 && sg * slot_rank(kind[j]) < sg * slot_rank(kind[j - 1]); --j) {
            const A ta = args[j]; args[j] = args[j - 1]; args[j - 1] = ta;
            const int tk = kind[j]; kind[j] = kind[j - 1]; kind[j - 1] = tk;
            const int tn = nblk[j]; nblk[j] = nblk[j - 1]; nblk[j - 1] = tn;
        }
}

// Blocks of the top (LIF [+ pred]) task: C = 8 one pixel per thread; C >= 16 the quad layout
// (lif_*_q_body), sized like a conv task so its blocks last about as long as theirs.
static int slot_top_blocks(int c, int B, int H, int W) {
    const int64_t npix = (int64_t)B * H * W;
    if (c < 16) return (int)((npix + 2 * NT - 1) / (2 * NT));
    const int64_t ppb = 2 * NT / (c / 4), target = snnflow_conv_blocks(B, H, W);
    const int64_t items = (npix + ppb * target - 1) / (ppb * target);
    return (int)((npix + ppb * items - 1) / (ppb * items));
}

// Tiles per block of the C = 8 forward tile pipeline (0: the one-tile-per-block body).  Default from
// SNNFLOW_PIPE_FWD at load time; snnflow_set_pipe overrides (A/B, tests).
static int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}
static int g_pipe_fwd = env_int("SNNFLOW_PIPE_FWD", 2);
// Block order of a C = 8 launch with pipelined tasks: 0 layer order, 1 pipelined tasks first, 2 last
static int g_pipe_order = env_int("SNNFLOW_PIPE_ORDER", 1);

// Blocks of a pipelined task: ceil(tiles / tpb), a multiple of 8 (block_tile's XCD groups).
static int pipe_blocks(int ntiles, int tpb) {
    const int nb = (ntiles + tpb - 1) / tpb;
    return (nb + 7) / 8 * 8;
}
// The DMA halo reads address a tensor through one buffer descriptor: 32-bit byte offsets.
static bool pipe_fits(int B, int H, int W, int c) { return (int64_t)B * H * W * c * 4 < ((int64_t)1 << 31); }

int snnflow_slot_supported(int c, int cin0) { return slot_c(c) && (cin0 == 2 || cin0 == 4) ? 1 : 0; }

// Block ranges of the tasks: each a multiple of 8 blocks (XCD grouping of block_tile).
static int slot_ranges(const int* nblk, int n, int* blk0) {
    int b = 0;
    for (int i = 0; i < n; ++i) {
        blk0[i] = b;
        b += (nblk[i] + 7) / 8 * 8;
    }
    return b;
}

int snnflow_fwd_slot(const snnflow_conv_fwd_args* conv, int nconv, const snnflow_lif_fwd_args* lif, void* stream) {
    const int nt = nconv + (lif ? 1 : 0);
    if (nconv < 0 || nt <= 0 || nt > kSlotTasks || (nconv && !conv)) SNN_FAIL(SNNFLOW_E_ARG, "fwd_slot: task count");
    FwdSlotParams p = {};
    const int c = nconv ? conv[0].c : lif->c;
    const int B = nconv ? conv[0].B : lif->B, H = nconv ? conv[0].H : lif->H, W = nconv ? conv[0].W : lif->W;
    if (!slot_c(c)) SNN_FAIL(SNNFLOW_E_CHANNELS, "fwd_slot: c must be 8, 16 or 32");
    for (int i = 0; i < nconv; ++i) {
        const snnflow_conv_fwd_args& a = conv[i];
        if (const int e = conv_fwd_check(&a)) return e;
        if (a.c != c || a.B != B || a.H != H || a.W != W) SNN_FAIL(SNNFLOW_E_ARG, "fwd_slot: tasks of different shapes");
        int kind;
        if (a.lif_in) {
            if (a.cin != c) SNN_FAIL(SNNFLOW_E_CHANNELS, "fwd_slot: lif_in requires cin == c");
            kind = a.wt_rec ? SK_LIF_REC : SK_LIF;
        } else if (a.wt_rec) {
            if (a.cin != c) SNN_FAIL(SNNFLOW_E_CHANNELS, "fwd_slot: recurrent cell requires cin == c");
            kind = SK_PLAIN_REC;
        } else if (a.cin == c) {
            kind = SK_PLAIN;
        } else if (a.cin == 1 || a.cin == 2 || a.cin == 4 || a.cin == 5) {
            kind = a.cin == 1 ? SK_HEAD1 : a.cin == 2 ? SK_HEAD2 : a.cin == 4 ? SK_HEAD4 : SK_HEAD5;
        } else {
            SNN_FAIL(SNNFLOW_E_CHANNELS, "fwd_slot: unsupported cin");
        }
        if (c != 8 && !(kind == SK_HEAD2 || kind == SK_HEAD4 || kind == SK_LIF || kind == SK_LIF_REC))
            SNN_FAIL(SNNFLOW_E_CHANNELS, "fwd_slot: c = 16 / 32 runs the LIFFireNet task kinds only");
        p.conv[i] = a;
        p.nblk[i] = snnflow_conv_blocks(B, H, W);
        if (c == 8 && g_pipe_fwd > 0 && (kind == SK_LIF || kind == SK_LIF_REC) && pipe_fits(B, H, W, c) &&
            !a.prev_spk_bits && !a.s_prev_bits)  // (the tile pipeline reads and writes fp32 spike planes only)
            kind = kind == SK_LIF ? SK_LIF_P : SK_LIF_REC_P;
        p.kind[i] = kind;
    }
    const int tpb = g_pipe_fwd;
    for (int i = 0; i < nconv; ++i) {
        if (p.kind[i] != SK_LIF_P && p.kind[i] != SK_LIF_REC_P) continue;
        const int nt = p.nblk[i];
        p.nblk[i] = pipe_blocks(nt, tpb);
        if (p.nblk[i] > (nt + 7) / 8 * 8) p.nblk[i] = (nt + 7) / 8 * 8;
    }
    if (lif) {
        if (const int e = lif_fwd_check(lif)) return e;
        if (lif->c != c || lif->B != B || lif->H != H || lif->W != W)
            SNN_FAIL(SNNFLOW_E_ARG, "fwd_slot: tasks of different shapes");
        if (c != 8 && !lif->pred_w) SNN_FAIL(SNNFLOW_E_CHANNELS, "fwd_slot: c = 16 / 32 top task needs the prediction");
        p.lif = *lif;
        p.kind[nconv] = lif->pred_w ? SK_TOP_PRED : SK_TOP;
        p.nblk[nconv] = slot_top_blocks(c, B, H, W);
    }
    if (c != 8) slot_sort(p.conv, p.kind, p.nblk, nconv);
    else if (SNNFLOW_SLOT_ORDER8) slot_sort(p.conv, p.kind, p.nblk, nconv, SNNFLOW_SLOT_ORDER8 == 2);
    else if (g_pipe_fwd > 0 && g_pipe_order) slot_sort(p.conv, p.kind, p.nblk, nconv, g_pipe_order == 2);
    p.ntask = nt;
    const int nb = slot_ranges(p.nblk, nt, p.blk0);
    const hipStream_t s = (hipStream_t)stream;
    if (c == 8) hipLaunchKernelGGL(k_fwd_slot<8>, dim3(nb), dim3(2 * NT), 0, s, p);
    else if (c == 16) hipLaunchKernelGGL(k_fwd_slot<16>, dim3(nb), dim3(2 * NT), 0, s, p);
    else hipLaunchKernelGGL(k_fwd_slot<32>, dim3(nb), dim3(2 * NT), 0, s, p);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_eval_slot(const snnflow_eval_fwd_args* tasks, int n, void* stream) {
    if (!tasks || n <= 0 || n > kEvalTasks) SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: task count");
    EvalSlotParams p = {};
    const int B = tasks[0].B, H = tasks[0].H, W = tasks[0].W;
    for (int i = 0; i < n; ++i) {
        const snnflow_eval_fwd_args& a = tasks[i];
        if (a.c != 8) SNN_FAIL(SNNFLOW_E_CHANNELS, "eval_slot: c must be 8");
        if (a.B != B || a.H != H || a.W != W || B <= 0 || H <= 0 || W <= 0)
            SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: tasks of different or empty shapes");
        if (a.n.bn_train) SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: BatchNorm in train mode needs batch statistics (snnflow_fwd_slot)");
        if (!a.state || !a.wt_ff || !a.n.bn_weight || !a.n.bn_bias || !a.n.running_mean || !a.n.running_var ||
            !a.n.beta || !a.n.threshold)
            SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: missing state, weights or neuron parameters");
        if (a.flow && (!a.pred_w || !a.pred_b)) SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: prediction without weights");
        if (!pipe_fits(B, H, W, 8)) SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: tensors of 2^31 bytes or more");
        const int ntiles = snnflow_conv_blocks(B, H, W);
        if (a.cin == a.c) {
            if (!a.s_in || !a.wt_ff_t) SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: spike input / fragment weights missing");
            if (a.s_prev && (!a.wt_rec || !a.wt_rec_t)) SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: recurrent weights missing");
            p.kind[i] = a.s_prev ? EK_REC : EK_FF;
            p.nblk[i] = pipe_blocks(ntiles, 2);
        } else if (a.cin == 2 || a.cin == 4) {
            if (!a.x || a.s_prev || a.flow) SNN_FAIL(SNNFLOW_E_ARG, "eval_slot: head task takes the event tensor only");
            p.kind[i] = a.cin == 2 ? EK_HEAD2 : EK_HEAD4;
            p.nblk[i] = ntiles;
        } else {
            SNN_FAIL(SNNFLOW_E_CHANNELS, "eval_slot: cin must be 2, 4 or c");
        }
        p.t[i] = a;
    }
    p.ntask = n;
    const int nb = slot_ranges(p.nblk, n, p.blk0);
    hipLaunchKernelGGL(k_eval_slot, dim3(nb), dim3(2 * NT), 0, (hipStream_t)stream, p);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_bwd_slot(const snnflow_layer_bwd_args* layer, int nlayer, const snnflow_lif_bwd_args* lif,
                     void* stream) {
    const int nt = nlayer + (lif ? 1 : 0);
    if (nlayer < 0 || nt <= 0 || nt > kSlotTasks || (nlayer && !layer)) SNN_FAIL(SNNFLOW_E_ARG, "bwd_slot: task count");
    BwdSlotParams p = {};
    const int c = nlayer ? layer[0].c : lif->c;
    const int B = nlayer ? layer[0].B : lif->B, H = nlayer ? layer[0].H : lif->H, W = nlayer ? layer[0].W : lif->W;
    if (!slot_c(c)) SNN_FAIL(SNNFLOW_E_CHANNELS, "bwd_slot: c must be 8, 16 or 32");
    for (int i = 0; i < nlayer; ++i) {
        const snnflow_layer_bwd_args& a = layer[i];
        if (const int e = layer_bwd_check(&a)) return e;
        if (a.c != c || a.B != B || a.H != H || a.W != W) SNN_FAIL(SNNFLOW_E_ARG, "bwd_slot: tasks of different shapes");
        int kind;
        if (a.lif_in) {
            if (a.cin != c) SNN_FAIL(SNNFLOW_E_CHANNELS, "bwd_slot: lif_in requires cin == c");
            if (c >= 16 && (!a.wd_ff || (a.wt_bwd_rec && a.g_state_prev && !a.wd_rec)))
                SNN_FAIL(SNNFLOW_E_ARG, "bwd_slot: c >= 16 needs the pre-split input-gradient fragments wd_ff / wd_rec");
            kind = a.wt_bwd_rec ? SK_LIF_REC : SK_LIF;
        } else if (a.wt_bwd_rec) {
            if (a.cin != c) SNN_FAIL(SNNFLOW_E_CHANNELS, "bwd_slot: recurrent cell requires cin == c");
            kind = SK_PLAIN_REC;
        } else if (a.cin == c) {
            kind = SK_PLAIN;
        } else if (a.cin == 2 || a.cin == 4) {
            kind = a.cin == 2 ? SK_HEAD2 : SK_HEAD4;
        } else {
            SNN_FAIL(SNNFLOW_E_CHANNELS, "bwd_slot: unsupported cin (2, 4 or c)");
        }
        if (c != 8 && !(kind == SK_HEAD2 || kind == SK_HEAD4 || kind == SK_LIF || kind == SK_LIF_REC))
            SNN_FAIL(SNNFLOW_E_CHANNELS, "bwd_slot: c = 16 / 32 runs the LIFFireNet task kinds only");
        // the fused weight gradients exist for the C = 8 LIF-fed tasks only: anywhere else the layer's
        // weight gradient would be silently lost
        // (ABI 40: and the feed-forward head tasks given their input x)
        const bool head_wg = (kind == SK_HEAD2 || kind == SK_HEAD4) && a.x != nullptr && !a.wslab_rec && !a.wt_bwd_rec;
        if ((a.wslab_ff || a.wslab_rec) && !(c == 8 && (kind == SK_LIF || kind == SK_LIF_REC)) && !head_wg)
            SNN_FAIL(SNNFLOW_E_ARG, "bwd_slot: wslab_ff / wslab_rec need a c = 8 LIF-fed task or a head task with x");
        p.layer[i] = a;
        p.kind[i] = kind;
        p.nblk[i] = layer_bwd_blocks(a);
    }
    if (lif) {
        if (const int e = lif_bwd_check(lif)) return e;
        if (lif->c != c || lif->B != B || lif->H != H || lif->W != W)
            SNN_FAIL(SNNFLOW_E_ARG, "bwd_slot: tasks of different shapes");
        if (lif->mem_grad_in) SNN_FAIL(SNNFLOW_E_ARG, "bwd_slot: mem_grad_in is a standalone-cell option");
        if (c != 8 && !lif->pred_w) SNN_FAIL(SNNFLOW_E_CHANNELS, "bwd_slot: c = 16 / 32 top task needs the prediction");
        p.lif = *lif;
        p.kind[nlayer] = lif->pred_w ? SK_TOP_PRED : SK_TOP;
        p.nblk[nlayer] = slot_top_blocks(c, B, H, W);
    }
    if (c != 8) {
        slot_sort(p.layer, p.kind, p.nblk, nlayer);
    } else if (SNNFLOW_SLOT_ORDER8) {
        slot_sort(p.layer, p.kind, p.nblk, nlayer, SNNFLOW_SLOT_ORDER8 == 2);
    }
    p.ntask = nt;
    const int nb = slot_ranges(p.nblk, nt, p.blk0);
    const hipStream_t s = (hipStream_t)stream;
    if (c == 8) hipLaunchKernelGGL(k_bwd_slot<8>, dim3(nb), dim3(2 * NT), 0, s, p);
    else if (c == 16) hipLaunchKernelGGL(k_bwd_slot<16>, dim3(nb), dim3(2 * NT), 0, s, p);
    else hipLaunchKernelGGL(k_bwd_slot<32>, dim3(nb), dim3(2 * NT), 0, s, p);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_set_pipe(int fwd_tiles_per_block, int bwd_tiles_per_block) {
    if (fwd_tiles_per_block < 0) SNN_FAIL(SNNFLOW_E_ARG, "set_pipe: negative tiles per block");
    if (bwd_tiles_per_block != 0) SNN_FAIL(SNNFLOW_E_ARG, "set_pipe: the backward runs one tile per block (ABI 38)");
    g_pipe_fwd = fwd_tiles_per_block;
    return 0;
}
int snnflow_get_pipe(int which) { return which == 0 ? g_pipe_fwd : 0; }

static int g_wg_bits = env_int("SNNFLOW_WG_BITS", 1);  // A/B: 0 = k_wgrad_bf32 / k_wgrad_bf on the bit planes
static int g_wg_head_sp2 = env_int("SNNFLOW_WG_HEAD_SP2", 1);
static bool wgrad_all_x_bits(const snnflow_wgrad_args* a) {
    for (int t = 0; t < a->nsteps; ++t)
        if (!a->steps[t].x_bits) return false;
    return true;
}

int snnflow_wgrad(const snnflow_wgrad_args* a, void* stream) {
    if (!a || a->B <= 0 || a->H <= 0 || a->W <= 0 || a->nsteps <= 0 || a->nsteps > SNNFLOW_MAX_WGRAD_STEPS ||
        !a->slab_ff || (a->rec && !a->slab_rec))
        SNN_FAIL(SNNFLOW_E_ARG, "wgrad: bad args");
    for (int t = 0; t < a->nsteps; ++t) {
        const snnflow_wgrad_step& st = a->steps[t];
        if (!st.g_cur || !st.y || !(st.x || st.x_bits) || (st.stats && !st.bnc)) SNN_FAIL(SNNFLOW_E_ARG, "wgrad: incomplete step");
        if ((st.x_bits || st.s_prev_bits) && !(a->exact_inputs && a->cin == a->c && (a->c == 8 || a->c == 16 || a->c == 32)))
            SNN_FAIL(SNNFLOW_E_ARG, "wgrad: spike bit planes need exact_inputs and cin == c in {8, 16, 32}");
        if (st.stats && !a->bn_weight) SNN_FAIL(SNNFLOW_E_ARG, "wgrad: BatchNorm step needs bn_weight");
    }
    const hipStream_t s = (hipStream_t)stream;
    const dim3 grid(snnflow_conv_blocks(a->B, a->H, a->W));
    const int c = a->c, cin = a->cin;
    if (!valid_c(c)) SNN_FAIL(SNNFLOW_E_CHANNELS, "wgrad: c must be 4, 8, 16 or 32");
#define WG_LAUNCH(CI_, CC_, REC_)                                                                          \
    do {                                                                                                   \
        constexpr int SP_ = (CC_ == 8 || CC_ == 16 || (CC_ == 32 && CI_ % 16 == 0)) ? 2 : 1;              \
        constexpr int SP2_ = (CC_ == 32 && CI_ == 2 && !REC_) ? 2 : SP_;                                  \
        if (SP2_ != SP_ && !g_wg_head_sp2)                                                                \
            hipLaunchKernelGGL((k_wgrad<CI_, CC_, REC_, SP_>), grid, dim3(NT * SP_), 0, s, *a);           \
        else                                                                                              \
            hipLaunchKernelGGL((k_wgrad<CI_, CC_, REC_, SP2_>), grid, dim3(NT * SP2_), 0, s, *a);         \
    } while (0)
#define WG_PICK(CI_, CC_)                                                                                  \
    do {                                                                                                   \
        if (a->rec) WG_LAUNCH(CI_, CC_, true);                                                             \
        else WG_LAUNCH(CI_, CC_, false);                                                                   \
    } while (0)
#define WG_CASE(CC_)                                                                                       \
    case CC_:                                                                                              \
        if (cin == CC_) WG_PICK(CC_, CC_);                                                                 \
        else if (cin == 1) WG_PICK(1, CC_);                                                                \
        else if (cin == 2) WG_PICK(2, CC_);                                                                \
        else if (cin == 3) WG_PICK(3, CC_);                                                                \
        else if (cin == 4) WG_PICK(4, CC_);                                                                \
        else if (cin == 5) WG_PICK(5, CC_);                                                                \
        else SNN_FAIL(SNNFLOW_E_CHANNELS, "wgrad: unsupported cin");                                       \
        break;
    if (a->exact_inputs && cin == c && (c == 8 || c == 16 || c == 32)) {
        const dim3 blk(NT * 2);
        if (c == 8) {
            if (a->rec) hipLaunchKernelGGL((k_wgrad_bf<8, true>), grid, blk, 0, s, *a);
            else hipLaunchKernelGGL((k_wgrad_bf<8, false>), grid, blk, 0, s, *a);
        } else if (c == 16) {
            if (a->rec) hipLaunchKernelGGL((k_wgrad_bf<16, true>), grid, blk, 0, s, *a);
            else hipLaunchKernelGGL((k_wgrad_bf<16, false>), grid, blk, 0, s, *a);
        } else if (g_wg_bits && wgrad_all_x_bits(a)) {
            // spike bit planes with the next step's loads in flight (k_wgrad_b32); recurrent layers as
            // two block sets (x and s_prev)
            hipLaunchKernelGGL(k_wgrad_b32, dim3(a->rec ? 2 * ((grid.x + 7) / 8 * 8) : grid.x), blk, 0, s, *a);
        } else {
            // feed-forward layers: k_wgrad_bf32 (two blocks per CU: 197 -> 164 us per cfg2 layer);
            // recurrent ones keep k_wgrad_bf (the split form's second staging pass measured 296 -> 315 us)
            if (a->rec) {
                if (SNNFLOW_WG32_SPLIT > 1) hipLaunchKernelGGL((k_wgrad_bf32<true>), grid, blk, 0, s, *a);
                else hipLaunchKernelGGL((k_wgrad_bf<32, true>), grid, blk, 0, s, *a);
            } else if (SNNFLOW_WG32_SPLIT) {
                hipLaunchKernelGGL((k_wgrad_bf32<false>), grid, blk, 0, s, *a);
            } else {
                hipLaunchKernelGGL((k_wgrad_bf<32, false>), grid, blk, 0, s, *a);
            }
        }
        SNN_CHECK_LAUNCH();
        return 0;
    }
    switch (c) {
        WG_CASE(4) WG_CASE(8) WG_CASE(16) WG_CASE(32)
        default: break;
    }
#undef WG_CASE
#undef WG_PICK
#undef WG_LAUNCH
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_slab_reduce(const snnflow_slab_desc* d, int n, int nblk, void* stream) {
    if (!d || n <= 0 || n > SNNFLOW_MAX_SLABS || nblk <= 0) SNN_FAIL(SNNFLOW_E_ARG, "slab_reduce: bad args");
    DescBatch<snnflow_slab_desc> batch = {};
    int maxe = 0;
    for (int i = 0; i < n; ++i) {
        batch.d[i] = d[i];
        if (!d[i].slab || !d[i].out || d[i].elems <= 0) SNN_FAIL(SNNFLOW_E_ARG, "slab_reduce: bad descriptor");
        maxe = d[i].elems > maxe ? d[i].elems : maxe;
    }
    hipLaunchKernelGGL(k_slab_reduce, dim3((maxe + SR_E - 1) / SR_E, n), dim3(SR_E * SR_G), 0, (hipStream_t)stream,
                       batch, nblk);
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"

namespace {
// Large-vector form (the U-Net's ~20 M parameters): per-block fp64 partial sums of squares in a
// fixed grid order, one block finishing the norm and the coefficient, a grid scaling the vector.
constexpr int CLIP2_NB = 512;

__global__ __launch_bounds__(256) void k_clip_partial(const float* __restrict__ g, int64_t n, double* partials) {
    __shared__ double part[4];
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double v = g[i];
        s += v * v;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (part[0] + part[1]) + (part[2] + part[3]);
}

__global__ void k_clip_coef(const double* partials, int nb, float max_norm, float eps, float* total_out, float* coef) {
    if (threadIdx.x != 0) return;
    double t = 0.0;
    for (int i = 0; i < nb; ++i) t += partials[i];
    const float total = (float)sqrt(t);
    const float c = max_norm / (total + eps);
    coef[0] = c < 1.0f ? c : 1.0f;
    if (total_out) total_out[0] = total;
}

__global__ __launch_bounds__(256) void k_clip_scale(float* __restrict__ g, int64_t n, const float* coef) {
    const float c = coef[0];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) g[i] = g[i] * c;
}
}  // namespace

extern "C" {

int snnflow_clip_grad_norm_large(float* g, int64_t n, float max_norm, float eps, float* total_out, double* scratch,
                                 void* stream) {
    if (!g || n < 0 || !scratch) SNN_FAIL(SNNFLOW_E_ARG, "clip_grad_norm_large: bad args");
    const hipStream_t s = (hipStream_t)stream;
    int64_t nb = (n + 255) / 256;
    if (nb > CLIP2_NB) nb = CLIP2_NB;
    if (nb < 1) nb = 1;
    float* coef = reinterpret_cast<float*>(scratch + CLIP2_NB);
    hipLaunchKernelGGL(k_clip_partial, dim3((unsigned)nb), dim3(256), 0, s, g, n, scratch);
    hipLaunchKernelGGL(k_clip_coef, dim3(1), dim3(64), 0, s, scratch, (int)nb, max_norm, eps, total_out, coef);
    int64_t gs = (n + 255) / 256;
    if (gs > 4096) gs = 4096;
    if (gs < 1) gs = 1;
    hipLaunchKernelGGL(k_clip_scale, dim3((unsigned)gs), dim3(256), 0, s, g, n, coef);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_clip_adam(const snnflow_clip_adam_args* a, void* stream) {
    if (!a || !a->grad || !a->exp_avg || !a->exp_avg_sq || !a->step || a->n < 0 || a->n > SNNFLOW_CLIP_ADAM_MAX_N ||
        a->ntensors < 0 || a->ntensors > SNNFLOW_ADAM_MAX_TENSORS)
        SNN_FAIL(SNNFLOW_E_ARG, "clip_adam: bad args (n <= SNNFLOW_CLIP_ADAM_MAX_N, ntensors <= SNNFLOW_ADAM_MAX_TENSORS)");
    for (int k = 0; k < a->ntensors; ++k) {
        const snnflow_adam_tensor& t = a->t[k];
        if (!t.param || t.offset < 0 || t.state_offset < 0 || t.numel < 0 || t.offset + t.numel > a->n)
            SNN_FAIL(SNNFLOW_E_ARG, "clip_adam: tensor range outside the flat buffer");
        if (k > 0 && t.offset < a->t[k - 1].offset + a->t[k - 1].numel)
            SNN_FAIL(SNNFLOW_E_ARG, "clip_adam: tensors must be in ascending, non-overlapping gradient order");
    }
    const hipStream_t s = (hipStream_t)stream;
    if (a->n <= CLIP_SLICE) {
        hipLaunchKernelGGL(k_clip_adam, dim3(1), dim3(CLIP_NT), 0, s, *a, 0);
    } else {
        const int nb = (int)((a->n + CLIP_SLICE - 1) / CLIP_SLICE);
        if (!a->scratch || nb > SNNFLOW_CLIP_SCRATCH) SNN_FAIL(SNNFLOW_E_ARG, "clip_adam: scratch needed above SNNFLOW_CLIP_ADAM_ONE_BLOCK");
        hipLaunchKernelGGL(k_clip_adam_norm, dim3(nb), dim3(CLIP_NT), 0, s, *a);
        hipLaunchKernelGGL(k_clip_adam, dim3(nb), dim3(CLIP_NT), 0, s, *a, nb);
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_clip_grad_norm(float* g, int64_t n, float max_norm, float eps, float* total_out, void* stream) {
    if (!g || n < 0) SNN_FAIL(SNNFLOW_E_ARG, "clip_grad_norm: bad args");
    hipLaunchKernelGGL(k_clip_grad_norm, dim3(1), dim3(CLIP_NT), 0, (hipStream_t)stream, g, n, max_norm, eps, total_out);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_lif_export(const float* x, const float* mem, const float* beta, const float* thr, int N, int C, int HW,
                       float* spk, float* mem_out, void* stream) {
    if (!x || !mem || !beta || !thr || !spk || !mem_out || N < 0 || C <= 0 || HW <= 0)
        SNN_FAIL(SNNFLOW_E_ARG, "lif_export: bad args");
    const int64_t total = (int64_t)N * C * HW;
    if (total == 0) return 0;
    int g = elem_grid(total);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_lif_export, dim3(g), dim3(NT), 0, (hipStream_t)stream, x, mem, beta, thr, total, C, HW, spk,
                       mem_out);
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
