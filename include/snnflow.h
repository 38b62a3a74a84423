/*
 * snnflow.h -- C-ABI of the MI355X-native LIFFireNet / event-warping hot path.
 *
 * Plain pointers (device memory, fp32 unless stated), sizes and a HIP stream.
 * No torch types.  Every entry point enqueues work on `stream` and returns
 * 0 on success, a negative SNNFLOW_E* code on bad arguments, or a positive
 * hipError_t; `snnflow_last_error()` describes the last failure (thread-local).
 * Nothing allocates or frees memory; all scratch is caller-provided, so every
 * call is capturable into a hipGraph.
 *
 * Layouts:
 *   activations  NHWC  [B][H][W][C]          (torch channels_last)
 *   cell state   [2][B][H][W][C]  (mem, spk)  (reference: torch.stack([mem, spk]))
 *   flow map     NCHW  [B][2][H][W]
 *   spike bits   [B][H][W] words of c bits (c = 8: uint8, 16: uint16, 32: uint32), ABI 39: channel ch
 *                of a pixel is bit (ch % 4) * (c / 4) + ch / 4 (SNNFLOW_SPK_BIT) -- an exact, 32x narrower
 *                copy of a spike plane (spikes are 0/1) that the wavefront forward writes and the
 *                recurrent convs and the deferred weight gradients read (c = 16 / 32)
 *   weights      torch [Cout][Cin][3][3]; kernels read the transposed copies made by
 *                snnflow_prep_weights.
 *
 * The reference has no native operators on this path (its only native op is the
 * forward-only CPU ONNX export op, ONNX_LIF_operator/src/lif_op.cpp:8-82); each entry
 * point below names the reference Python it replaces.
 */
#ifndef SNNFLOW_H
#define SNNFLOW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SNNFLOW_ABI_VERSION 40

#define SNNFLOW_E_ARG (-1)      /* invalid argument / unsupported shape */
#define SNNFLOW_E_CHANNELS (-2) /* channel count without a compiled kernel */

/* Tile geometry of the conv kernels (block = SNNFLOW_TILE_H x SNNFLOW_TILE_W pixels). */
#define SNNFLOW_TILE_H 8
#define SNNFLOW_TILE_W 32

/* Per-layer neuron + BatchNorm parameters
 * (SNNtorch_spiking_submodules.py:230-251 / :451-475: bn = BatchNorm2d(C, 0.1, 1e-5),
 *  lif = snn.Leaky(beta, threshold, reset_mechanism, reset_delay=False)). */
typedef struct snnflow_neuron {
    const float* bn_weight;     /* [C] gamma                                   */
    const float* bn_bias;       /* [C]                                          */
    float* running_mean;        /* [C] updated in place when bn_train          */
    float* running_var;         /* [C]                                          */
    int64_t* num_batches_tracked; /* [1] incremented when bn_train (may be NULL) */
    const float* beta;          /* [C] lif.beta (clamped to [0,1] on use)       */
    const float* threshold;     /* [C] lif.threshold (clamp_min 0.01 done by prep) */
    double momentum, eps;
    int bn_train;               /* 1: batch statistics (train), 0: running stats */
    int zero_reset;             /* 1: reset_mechanism="zero", 0: "subtract"     */
} snnflow_neuron;

/* ---- weight preparation -------------------------------------------------
 * Transposes a conv weight [C][Cin][3][3] into wt_fwd [3][3][Cin][C] and
 * wt_bwd [3][3][C][Cin] (skipped when w == NULL); if threshold != NULL clamps its
 * first c entries in place to >= 0.01
 * (SNNtorch_spiking_submodules.py:284 / :516 `threshold.data.clamp_(min=0.01)`). */
int snnflow_prep_weights(const float* w, int c, int cin, float* wt_fwd, float* wt_bwd,
                         float* threshold, void* stream);

/* All layers' weight preparation in one launch (one descriptor per conv weight and/or
 * threshold vector; the fields mean what the snnflow_prep_weights arguments mean,
 * thr_n = entries of `threshold` to clamp).  n <= SNNFLOW_MAX_BATCH. */
typedef struct snnflow_prep_desc {
    const float* w; int c, cin; float* wt_fwd; float* wt_bwd;
    float* threshold; int thr_n;
    /* ABI 15, optional (NULL = skip; cin == c, c % 8 == 0): the weights split into three bf16
     * parts (hi + mid + lo == w exactly) in the matrix-core operand order of the kernels --
     * frag_fwd for the forward conv (snnflow_conv_fwd_args.wf_ff / wf_rec), frag_bwd for the
     * input-gradient conv (snnflow_layer_bwd_args.wd_ff / wd_rec); snnflow_frag_halfs(c, cin)
     * bf16 values (uint16 bit patterns) each */
    uint16_t* frag_fwd; uint16_t* frag_bwd;
    /* ABI 29, optional: zero_n doubles at `zero` are set to 0 (the batch-sum accumulators of the
     * following forward / backward pass ride along with the weight preparation: one launch fewer
     * than a separate fill).  A descriptor may carry only this (w = threshold = NULL). */
    double* zero; int64_t zero_n;
} snnflow_prep_desc;
int snnflow_frag_halfs(int c, int cin);
#define SNNFLOW_MAX_BATCH 16
int snnflow_prep_weights_batch(const snnflow_prep_desc* d, int n, void* stream);

/* Batch-statistics accumulators.  BatchNorm in train mode needs sums over (B,H,W)
 * between the producing conv and the consuming LIF.  Each producer block adds its
 * partial sums with fp64 atomics into one of SNNFLOW_ACC_SHARDS replicas of the
 * accumulator (replica = block index mod shards: 512 blocks adding into one address
 * serialise at the memory-side atomic unit); the next kernel in the chain sums the
 * replicas in its prologue and derives the statistics.  An accumulator of n sums
 * occupies SNNFLOW_ACC_LEN(n) doubles ([shard][SNNFLOW_ACC_STRIDE(n)]).  It must be
 * zero when its producer starts: kernels zero the accumulators named in
 * `zero0`/`zero1` (`zero_n` doubles each), which the caller chooses among
 * accumulators already consumed by an earlier kernel of the chain. */
#define SNNFLOW_ACC_SHARDS 32
#define SNNFLOW_ACC_STRIDE(n) ((((n) + 15) / 16) * 16)
#define SNNFLOW_ACC_LEN(n) (SNNFLOW_ACC_SHARDS * SNNFLOW_ACC_STRIDE(n))

/* ---- forward: [LIF of layer l on a halo tile] + conv3x3(layer l+1) [+ BN batch sums]
 * Replaces, per time step, `lif(bn(...))` of layer l fused with `ff(input_)`
 * [+ `rec(prev_spk)`] of layer l+1 and the batch-sum part of its `bn`
 * (SNNtorch_spiking_submodules.py:289-305 and :521-550).
 * lif_in = 0: x is a strided tensor (e.g. event_cnt NCHW) with cin channels.
 * lif_in = 1: the input spikes are computed from the previous layer's pre-BN conv
 *             output prev_y (NHWC), its membrane prev_mem (NULL = zeros) and its batch
 *             sums prev_acc (SNNFLOW_ACC_LEN(2cin), train) or running stats (eval); block 0 writes
 *             prev_stats [2][cin] (mean, invstd) and updates the running statistics;
 *             prev_state [2][B][H][W][cin] receives (mem_out, spk) of the previous layer. */
typedef struct snnflow_conv_fwd_args {
    int B, H, W, cin, c;
    int lif_in;
    const float* x; int64_t xs_b, xs_c, xs_h, xs_w;   /* lif_in == 0 */
    const float* prev_y; const float* prev_mem;        /* lif_in == 1 */
    const double* prev_acc; float* prev_stats;
    snnflow_neuron prev; float* prev_state;
    const float* wt_ff;         /* [3][3][cin][c]                      */
    const float* wt_rec;        /* [3][3][c][c] or NULL (feed-forward) */
    /* the same weights in the backward layout ([3][3][c][cin], [3][3][c][c]): the matrix-core
     * (MFMA) B operand of the cin == c kernels, required there (wt_rec_t iff wt_rec) */
    const float* wt_ff_t; const float* wt_rec_t;
    const float* s_prev;        /* NHWC [B][H][W][c] previous-step spikes; NULL = zeros */
    float* y;                   /* out NHWC [B][H][W][c] pre-BN current           */
    double* acc;                /* += SNNFLOW_ACC_LEN(2c) (sum y, sum y^2); NULL = no batch sums (eval) */
    double* zero0; double* zero1; int zero_n;
    /* ABI 15, optional: bf16 fragments of wt_ff_t / wt_rec_t (snnflow_prep_desc.frag_fwd) for the
     * spike convs of the cin == c kernels at c = 16, 32 (else split in the kernel) */
    const uint16_t* wf_ff; const uint16_t* wf_rec;
    /* ABI 33: 1 = store only the membrane half of prev_state (a caller whose spike half is never read:
     * a feed-forward layer's intermediate time steps in a window -- the backward recomputes the spikes) */
    int state_spk_skip;
    /* ABI 39, optional (lif_in = 1, cin == c in {8, 16, 32}; not the c = 8 tile pipeline): prev_spk_bits
     * receives the spike bit plane of the previous layer (the spikes the LIF of this task computes; interior
     * pixels of every tile, i.e. every pixel); s_prev_bits, if set, replaces s_prev (the previous-step spikes
     * of this layer as a bit plane: exact 0/1 by construction) */
    uint8_t* prev_spk_bits; const uint8_t* s_prev_bits;
} snnflow_conv_fwd_args;
int snnflow_conv_fwd(const snnflow_conv_fwd_args* a, void* stream);
int snnflow_conv_blocks(int B, int H, int W);

/* ---- forward: LIF of a layer [+ pred ConvLayer(C->2,1x1,bias)+tanh]
 * Replaces `lif(bn(.))` (SNNtorch_spiking_submodules.py:293-320) and
 * `pred` (models/submodules.py:96-113, models/model.py:182). */
typedef struct snnflow_lif_fwd_args {
    int B, H, W, c;
    const float* y; const float* mem;
    const double* acc;          /* SNNFLOW_ACC_LEN(2c) batch sums (train) */
    float* stats;               /* out [2][c] (mean, invstd) */
    snnflow_neuron n; float* state;
    const float* pred_w;        /* [2][c] or NULL (no pred) */
    const float* pred_b;        /* [2] */
    float* flow;                /* NCHW [B][2][H][W] */
    double* zero0; double* zero1; int zero_n;
    int state_spk_skip;         /* ABI 33: 1 = store only the membrane half of state (as snnflow_conv_fwd_args) */
} snnflow_lif_fwd_args;
int snnflow_lif_fwd(const snnflow_lif_fwd_args* a, void* stream);

/* Gradient destinations of one layer's neuron parameters (fp32, [C] each). */
typedef struct snnflow_neuron_grad {
    float* bn_weight; float* bn_bias; float* beta; float* threshold;
} snnflow_neuron_grad;

/* Number of doubles of a backward accumulator for c channels (3c LIF/BN sums + 2c+2 pred). */
/* Bit of channel ch in a pixel word of a c-channel spike bit plane (ABI 39). */
#define SNNFLOW_SPK_BIT(c, ch) (((ch) % 4) * ((c) / 4) + (ch) / 4)

#define SNNFLOW_BWD_ACC(c) (5 * (c) + 2) /* sums per layer; storage SNNFLOW_ACC_LEN(SNNFLOW_BWD_ACC(c)) */

/* ---- backward of the top layer: [pred backward] + LIF/ATan surrogate backward
 * g_s = g_out + g_state_spk + pred_w^T (g_flow * (1 - flow^2)); g_v = g_s * sg(v - theta).
 * Writes g_cur (= dL/d BN-output, NHWC) [and g_mem = dL/d membrane input] and adds
 * (sum g, sum (y-mean) g, sum g*m') [and the pred weight/bias sums] into acc. */
typedef struct snnflow_lif_bwd_args {
    int B, H, W, c;
    const float* y; const float* mem; const float* stats; snnflow_neuron n;
    const float* g_out;         /* NHWC grad of the spike output or NULL          */
    const float* g_state;       /* [2][B][H][W][c] grad of the state output or NULL */
    const float* pred_w; const float* flow; const float* g_flow;  /* pred or NULL    */
    int64_t gflow_sb, gflow_sc; /* element strides of g_flow (batch, channel); HW dense */
    float* g_cur;
    float* g_mem;               /* NHWC grad of the membrane input (beta*(1-r)*g_v) or NULL */
    double* acc;                /* += SNNFLOW_BWD_ACC(c) sums (storage SNNFLOW_ACC_LEN of it) */
    double* zero0; double* zero1; int zero_n;
    /* 1: the membrane half of g_state carries gradient (cells with detach=False,
     * SNNtorch_spiking_submodules.py:309-311: mem_out = v - (s - r)*v | v - (s - r)*theta is not
     * detached); its threshold part sum g_mo*(1 - s + r) goes to acc[3c + ch].  No prediction. */
    int mem_grad_in;
} snnflow_lif_bwd_args;
int snnflow_lif_bwd(const snnflow_lif_bwd_args* a, void* stream);

/* ---- backward of one layer on the critical path: BN backward + conv dgrad of layer l
 * [+ LIF backward of layer l-1 on the dgrad result] (the reverse of snnflow_conv_fwd).
 * Block 0 turns acc_in into layer l's neuron-parameter gradients (and pred gradients
 * when has_pred), written (accumulate=0) or added, and stores the BatchNorm backward
 * coefficients of this layer-step in bnc_out for the deferred weight gradient
 * (snnflow_wgrad). */
typedef struct snnflow_layer_bwd_args {
    int B, H, W, cin, c;
    const float* y; const float* stats; const float* g_cur;
    const double* acc_in;       /* SNNFLOW_BWD_ACC(c) sums of layer l's LIF backward */
    snnflow_neuron n;           /* BN / neuron parameters of layer l */
    snnflow_neuron_grad ng;
    int has_pred; float* g_pred_w; float* g_pred_b;
    int accumulate;
    float* bnc_out;             /* [2][c] (grad_mean, k) of layer l's BN backward */
    const float* wt_bwd_ff;     /* [3][3][c][cin]  (NULL: no input gradient)        */
    const float* wt_bwd_rec;    /* [3][3][c][c] or NULL                             */
    /* the same weights in the forward layout ([3][3][cin][c], [3][3][c][c]): MFMA B operand of
     * the input-gradient convs of the cin == c kernels, required there with their wt_bwd_* */
    const float* wt_fwd_ff; const float* wt_fwd_rec;
    int lif_in;
    float* g_x; int64_t gxs_b, gxs_c, gxs_h, gxs_w;   /* lif_in=0: input gradient (strided) or NULL */
    float* g_state_prev;        /* [2][B][H][W][c] grad of the previous state (rec) or NULL */
    int zero_mem_half;          /* 1: also zero-fill the membrane half of g_state_prev */
    /* lif_in = 1: LIF backward of layer l-1 */
    const float* prev_y; const float* prev_mem; const float* prev_stats; snnflow_neuron prev;
    const float* prev_g_state;  /* [2][B][H][W][cin] or NULL */
    float* prev_g_cur; float* prev_g_mem;
    double* acc_out;            /* += SNNFLOW_BWD_ACC(cin) sums for layer l-1 */
    double* zero0; double* zero1; int zero_n;
    /* ABI 15, optional: bf16 fragments of wt_fwd_ff / wt_fwd_rec (snnflow_prep_desc.frag_bwd)
     * for the input-gradient convs of the cin == c kernels at c = 16, 32 (else f32 matrix cores) */
    const uint16_t* wd_ff; const uint16_t* wd_rec;
    /* ABI 23, optional: the layer's weight gradients fused into this backward task (lif_in = 1,
     * c = cin = 8, wavefront launches only -- snnflow_bwd_slot; the single-task call ignores them).
     * The task already holds G = dL/dy of its tile with the halo (BN backward applied) and
     * recomputes layer l-1's spikes x of its tile for the LIF backward, so
     *   dW_ff[co][ci][k] += sum_{q in tile} x[q][ci] G[q - k][co]     (= sum_p G[p][co] x[p + k][ci])
     * and, with s_prev (NHWC [B][H][W][c] spikes of layer l at the previous step; NULL: zero state),
     *   dW_rec[co][ci][k] += sum_{q in tile} s_prev[q][ci] G[q - k][co]
     * go to the block's row of wslab_ff / wslab_rec ([snnflow_conv_blocks()][c*cin*9], the
     * deferred path's slab layout): written (wslab_accumulate = 0) or added.  Rows are per tile and
     * every (layer, step) task of a pass runs in its own launch, so the accumulation over the steps
     * is a fixed-order read-modify-write (deterministic); snnflow_slab_reduce sums the rows. */
    float* wslab_ff; float* wslab_rec; const float* s_prev; int wslab_accumulate;
    /* ABI 40, optional: the head's weight gradient fused into its backward task (lif_in = 0, cin 2 or 4,
     * no recurrent conv, wavefront launches only).  The head task holds G = dL/dy of its tile after
     * the BN backward and nothing else reads it, so with wslab_ff and x (the layer input, strided as
     * g_x: [B][cin][H][W] at xs_b, xs_c, xs_h, xs_w)
     *   dW_ff[co][ci][k] += sum_p G[p][co] x[p + k][ci]
     * goes to the block's row of wslab_ff (written or added as above; the deferred path's per-tile
     * per-step order of snnflow_wgrad's vector kernel, one step per call). */
    const float* x; int64_t xs_b, xs_c, xs_h, xs_w;
} snnflow_layer_bwd_args;
int snnflow_layer_bwd(const snnflow_layer_bwd_args* a, void* stream);

/* ---- wavefront launches (ABI 14) -------------------------------------------
 * Up to SNNFLOW_MAX_SLOT_TASKS mutually independent layer-steps of one model in ONE launch.
 * A single layer-step launch is latency-bound (load -> LIF -> conv -> store chain of one
 * block per tile); the (layer, step) grid of a T-step sequence instead runs as 2(T-1)+L+1
 * launches of about (L+1)/2 layer-steps each (task (l, t) in launch l + 2t; snnflow/engine.py
 * FireNetSequence).  Each task means exactly what the single-task call with the same
 * arguments means; the caller guarantees that no task reads what another task of the same
 * launch writes.  Forward: conv tasks (snnflow_conv_fwd) + at most one LIF(+pred) task
 * (snnflow_lif_fwd); backward: layer tasks (snnflow_layer_bwd) + at most one top-LIF task
 * (snnflow_lif_bwd).  All tasks of a launch share c and B, H, W.
 * snnflow_slot_supported(c, cin0): 1 if both slot kernels take every task of a model with
 * c channels and a cin0-channel input (c = 8; cin0 2 or 4), else 0 (C = 16 / 32: one
 * layer-step already fills the chip). */
#define SNNFLOW_MAX_SLOT_TASKS 4
int snnflow_fwd_slot(const snnflow_conv_fwd_args* conv, int nconv, const snnflow_lif_fwd_args* lif,
                     void* stream);
int snnflow_bwd_slot(const snnflow_layer_bwd_args* layer, int nlayer, const snnflow_lif_bwd_args* lif,
                     void* stream);
int snnflow_slot_supported(int c, int cin0);
/* Tuning (ABI 27): tiles per block of the c = 8 LIF-fed forward tasks of the wavefront launches
 * (0: one tile per block; >= 1: the tile pipeline, which overlaps the next tile's halo loads by
 * LDS-DMA with this tile's math).  Process-wide; default from SNNFLOW_PIPE_FWD at load time.  Results
 * do not depend on it beyond fp64-atomic summation order.  ABI 38: the backward runs one tile per
 * block only -- bwd_tiles_per_block must be 0 (its tile pipeline measured slower and was removed);
 * snnflow_get_pipe(0) reads the forward value, snnflow_get_pipe(1) is 0. */
int snnflow_set_pipe(int fwd_tiles_per_block, int bwd_tiles_per_block);
int snnflow_get_pipe(int which);

#define SNNFLOW_MAX_LAYERS 8   /* cells of a LIFFireNet-family model (the step driver's plan) */

/* ---- deferred weight gradients of one layer over many time steps ----------
 * Nothing on the backward chain depends on dW, so the weight gradients of a layer
 * are computed once per backward pass over all its time steps:
 *   dW_ff[co][ci][k]  = sum_t sum_p G_t[p][co] x_t[p + k][ci]
 *   dW_rec[co][ci][k] = sum_t sum_p G_t[p][co] s_prev_t[p + k][ci]
 * with G_t = ((g_cur - grad_mean) - (y - mean) k) invstd gamma (BN backward, from the
 * coefficients layer_bwd stored in bnc).  One block per tile accumulates over the
 * steps in registers and writes (accumulate=0) or adds its per-block slab once;
 * snnflow_slab_reduce sums the slabs.  Up to SNNFLOW_MAX_WGRAD_STEPS steps per call. */
typedef struct snnflow_wgrad_step {
    const float* g_cur;         /* NHWC [B][H][W][c] */
    const float* y;             /* NHWC pre-BN conv output */
    const float* x; int64_t xs_b, xs_c, xs_h, xs_w;   /* ff conv input (strided) */
    const float* s_prev;        /* NHWC previous-step spikes (rec conv input) or NULL */
    const float* stats;         /* [2][c] mean, invstd; NULL: no BatchNorm (G = g_cur, ConvLIF) */
    const float* bnc;           /* [2][c] grad_mean, k (ignored without stats) */
    /* ABI 39, optional (cin == c in {16, 32}, exact_inputs): x / s_prev as spike bit planes (replace them) */
    const uint8_t* x_bits; const uint8_t* s_prev_bits;
} snnflow_wgrad_step;
#define SNNFLOW_MAX_WGRAD_STEPS 32
typedef struct snnflow_wgrad_args {
    int B, H, W, cin, c, nsteps, accumulate, rec;
    int exact_inputs;           /* 1: every x and s_prev value is exact in bf16 (spikes):
                                   cin == c layers then run on the bf16 matrix cores */
    const float* bn_weight;     /* [c] gamma (ignored without stats) */
    float* slab_ff;             /* snnflow_conv_blocks() x c*cin*9 */
    float* slab_rec;            /* snnflow_conv_blocks() x c*c*9 (rec layers) */
    snnflow_wgrad_step steps[SNNFLOW_MAX_WGRAD_STEPS];
} snnflow_wgrad_args;
int snnflow_wgrad(const snnflow_wgrad_args* a, void* stream);

/* ---- U-Net neuron flavour: ConvLIF / ConvLIFRecurrent ----------------------
 * models/spiking_submodules.py:121-151 (ConvLIF, stride 1), :265-300 (ConvLIFRecurrent):
 *   I = conv_ff(x) [+ conv_rec(z_prev)];  leak = sigmoid(leak_raw);  th = clamp_min(thresh, 0.01)
 *   hard: v_out = v*leak*(1 - z) + (1 - leak)*I    soft: v_out = v*leak + (1 - leak)*I - z*th
 *   z_out = (v_out - th > 0); backward of the spike: g / (1 + width*(v_out - th)^2) (ArctanSpike,
 *   models/spiking_util.py:82-109); z (reset) detached, v not (BPTT through the membrane).
 * No normalisation; weights prepared by snnflow_prep_weights.  The weight gradients come from
 * snnflow_wgrad with stats = NULL (G = g_current). */
typedef struct snnflow_convlif_params {
    const float* leak;          /* [c] raw leak parameter */
    const float* thresh;        /* [c] raw threshold */
    float act_width;
    int hard_reset;
} snnflow_convlif_params;

typedef struct snnflow_convlif_fwd_args {
    int B, H, W, cin, c;
    const float* x; int64_t xs_b, xs_c, xs_h, xs_w;   /* input (strided) */
    const float* prev_state;    /* [2][B][H][W][c] (v, z) or NULL (zeros) */
    const float* wt_ff;         /* [3][3][cin][c] */
    const float* wt_rec;        /* [3][3][c][c] (ConvLIFRecurrent) or NULL */
    snnflow_convlif_params p;
    const float* residual; int64_t rs_b, rs_c, rs_h, rs_w;   /* added to the spikes, or NULL */
    float* out;                 /* NHWC z_out + residual */
    float* state;               /* [2][B][H][W][c] (v_out, z_out) */
    float* current;             /* NHWC I, saved for the backward pass */
} snnflow_convlif_fwd_args;
int snnflow_convlif_fwd(const snnflow_convlif_fwd_args* a, void* stream);

typedef struct snnflow_convlif_bwd_args {
    int B, H, W, cin, c;
    const float* g_out; int64_t gs_b, gs_c, gs_h, gs_w;   /* grad of out (strided) or NULL */
    const float* g_state;       /* [2][B][H][W][c] grad of (v_out, z_out) or NULL */
    const float* state;         /* the forward's state output */
    const float* prev_state;    /* [2][B][H][W][c] or NULL */
    const float* current;       /* the forward's current */
    const float* wt_bwd_ff;     /* [3][3][c][cin] or NULL (no input gradient) */
    const float* wt_bwd_rec;    /* [3][3][c][c] or NULL */
    snnflow_convlif_params p;
    float* g_x; int64_t gxs_b, gxs_c, gxs_h, gxs_w;   /* or NULL */
    float* g_prev;              /* [2][B][H][W][c] grad of prev_state or NULL */
    float* g_current;           /* NHWC dL/dI (input of snnflow_wgrad) */
    double* acc;                /* += SNNFLOW_ACC_LEN(2c): sum dL/dth, sum dL/dleak (must start zeroed) */
} snnflow_convlif_bwd_args;
int snnflow_convlif_bwd(const snnflow_convlif_bwd_args* a, void* stream);

/* Parameter gradients from the backward sums: g_thresh = sum * (thresh >= 0.01) (clamp_min),
 * g_leak = sum * s * (1 - s), s = sigmoid(leak) (written, or added when accumulate). */
int snnflow_convlif_param_grads(const double* acc, const float* leak, const float* thresh, int c, int accumulate,
                                float* g_leak, float* g_thresh, void* stream);

/* ---- on-device event encodings (dataloader/encodings.py:30-85, dataloader/base.py) ----
 * Event e of sample b has fields ts/ys/xs/ps at base + b*batch_stride + e*ev_stride
 * (ev_stride 4 for an event list [B][N][4] (ts, y, x, p), 1 for separate arrays).
 * Pixel = (long)y * W + (long)x (truncation, as .long()); events outside the sensor are
 * skipped (the reference's index_put_ would raise).  Outputs (any may be NULL) are fully
 * written:
 *   cnt      [B][2][H][W]   events_to_channels: += p*p into channel 0 (p >= 0) / 1 (p <= 0)
 *   voxel    [B][bins][H][W] events_to_voxel: t = ts*(bins-1) [rounded half-even], += p*max(0, 1-|t-k|)
 *   image    [B][H][W]      events_to_image(ps, accumulate) (accumulate=0: last write wins)
 *   mask     [B][1][H][W]   events_to_image(|p|, accumulate=False)  (create_mask_encoding)
 *   pol_mask [B][N][2]      create_polarity_mask: (p<0 ? 0 : p, -(p>0 ? 0 : p)) */
typedef struct snnflow_encode_args {
    int B, N, H, W;
    const float* ts; const float* ys; const float* xs; const float* ps;
    int64_t ev_stride, batch_stride;
    int num_bins, round_ts, accumulate;
    float* cnt; float* voxel; float* image; float* mask; float* pol_mask;
} snnflow_encode_args;
int snnflow_encode_events(const snnflow_encode_args* a, void* stream);

/* Sums per-block weight-gradient slabs: out[i][e] = sum_b slab[i][b][e]. */
typedef struct snnflow_slab_desc { const float* slab; float* out; int elems; } snnflow_slab_desc;
#define SNNFLOW_MAX_SLABS 16
int snnflow_slab_reduce(const snnflow_slab_desc* d, int n, int nblk, void* stream);

/* ---- event warping / contrast-maximisation loss (loss/flow.py:178-303) ----
 * Window k's events are the concatenated index range [off[k], off[k+1]) of every sample
 * (flow.py:58-121); its timestamps are ts + k (flow.py:92).  Each window's tensors are
 * passed by pointer (tables below), so nothing is concatenated on the device. */
#define SNNFLOW_MAX_WINDOWS 64
typedef struct snnflow_iwe_loss_args {
    int B, M, T, H, W;
    int tf;                     /* flow/mask windows: T, or 1 when overwrite_intermediate
                                   (all events use the last flow; loss/flow.py:123-150) */
    /* per event window k < T (N_k = off[k+1] - off[k] events per sample, M = sum N_k):
     * events [B][N_k][4] (ts, y, x, p) and polarity masks [B][N_k][2] -- the tensors
     * event_flow_association recorded, read in place (no concatenation) */
    const float* events[SNNFLOW_MAX_WINDOWS]; const float* pol[SNNFLOW_MAX_WINDOWS];
    /* per flow window t < tf: flow [B][2][H][W] and event mask [B][H][W] */
    const float* flows[SNNFLOW_MAX_WINDOWS]; const float* masks[SNNFLOW_MAX_WINDOWS];
    int32_t off[SNNFLOW_MAX_WINDOWS + 1];  /* pass offsets off[0..T], by value */
    float flow_scaling, weight;
    int smoothing_mask, overwrite_intermediate, loss_scaling;
    float* images;              /* 16-B aligned scratch of snnflow_iwe_scratch_floats(B, M, T, tf, H, W)
                                   floats: the IWEs [2 dir][4 img][B][H*W] (cnt+, cnt-, ts+, ts-),
                                   then the events binned by warped band (forward) and by own-pixel
                                   band (backward) -- ABI 38; kept from the forward to the backward */
    double* acc;                /* scratch snnflow_iwe_acc_doubles(B, H, W, tf): per-block partial
                                   sums, reduced in a fixed order (deterministic loss) */
    float* persample;           /* scratch [2 dir][B][4]: S+, S-, nz, loss_b          */
    float* smooth;              /* scratch [8]                                         */
    float* loss;                /* out [1]                                             */
} snnflow_iwe_loss_args;
int snnflow_iwe_loss_fwd(const snnflow_iwe_loss_args* a, void* stream);
/* g_loss: device scalar; g_flows out [B][tf][2][H][W] (fully written).  Reads the forward's images
 * scratch (the IWEs and, ABI 38, the events binned by the pixel band of their own pixel -- formed by the
 * forward when tf == T, here otherwise); one block per (sample, flow window, band) forms the smoothness
 * gradient of its pixels and the events' flow gradients (the image gradients formed at their warped
 * corners), summed per pixel in exact two-word fixed point (order-independent: bit-reproducible
 * g_flows), and writes the band once.  H * W <= 2^21, W <= 1791. */
int snnflow_iwe_loss_bwd(const snnflow_iwe_loss_args* a, const float* g_loss, float* g_flows, void* stream);
int snnflow_iwe_acc_doubles(int B, int H, int W, int tf);
/* ABI 39: device-side argument faults the kernels detected and skipped instead of reading out of bounds
 * (bit 1: a forward bin segment outside its window's records, k_iwe_splat; bit 2: the same in the
 * backward, k_iwe_bwd_band -- a corrupted or stale images scratch).  Synchronises the device; clear != 0
 * resets the flags.  Returns the flag bits (>= 0) or an error code.  (Diagnostics: SNNFLOW_FAULT_INJECT=1 / 2
 * at library load corrupts one bin-table entry before k_iwe_splat / k_iwe_bwd_band, for tests.) */
int snnflow_device_errors(int clear);
/* floats of the images scratch (ABI 38: the IWEs and both binnings of the events; H * W <= 2^21) */
int64_t snnflow_iwe_scratch_floats(int B, int M, int T, int tf, int H, int W);

/* utils/iwe.py:20-71 get_interpolation (+ purge_unfeasible :4-17) for one pass:
 * idx out [B][K*M] int32 (corner-major, K=4 bilinear / 1 rounded), w out [B][K*M]. */
int snnflow_iwe_corners(const float* events, const float* flow_ev, int B, int M, float tref,
                        int H, int W, float flow_scaling, int round_idx, int32_t* idx, float* w,
                        void* stream);
/* utils/iwe.py:74-93 interpolate: img[b][idx] += w * pol (img zeroed by the call). */
int snnflow_iwe_interpolate(const int32_t* idx, const float* w, const float* pol, int64_t pol_sb,
                            int B, int K, int H, int W, float* img, void* stream);
/* Autograd of the two above (the reference's weights carry gradient, utils/iwe.py:59, 65, 91):
 * corners_bwd: g_w [B][4*M] (corner-major, bilinear only) -> g_flow_ev [B][M][2] (y, x), overwritten;
 * interpolate_bwd: g_img [B][H*W] -> g_w [B][K] = g_img[b][idx] * pol, overwritten. */
int snnflow_iwe_corners_bwd(const float* events, const float* flow_ev, int B, int M, float tref,
                            int H, int W, float flow_scaling, const float* g_w, float* g_flow_ev,
                            void* stream);
int snnflow_iwe_interpolate_bwd(const int32_t* idx, const float* pol, int64_t pol_sb, int B, int K,
                                int H, int W, const float* g_img, float* g_w, void* stream);

/* ---- evaluation path (eval_flow.py:220-282, utils/iwe.py:96-150, loss/flow.py:597-649) ----
 * deblur_events / compute_pol_iwe: per event gather the flow at its pixel ((long)(y*W + x)),
 * warp to tref, round half-even (round_idx) or take the 4 bilinear corners, purge
 * out-of-sensor locations, and scatter weight * mask into nimg images of out
 * [B][nimg][H][W] (fully written).  Mask of image k: pol[e*pol_stride + k], or 1 when pol
 * is NULL (nimg = 1 only). */
int snnflow_pol_iwe(const float* events, const float* flow, const float* pol, int64_t pol_stride, int nimg, int B,
                    int N, int H, int W, float tref, float flow_scaling, int round_idx, float* out, void* stream);

/* AEE: flow' = (flow * flow_scaling) * dt_ratio[b]; error = |flow' - gt|_2 per pixel;
 * valid = event_mask && gt != (0,0); AEE[b] = sum(error*valid) / (sum(valid) + 1e-9);
 * outliers = (error*valid > 3) && (error*valid > 0.05*|flow'|*valid), counted over the
 * whole batch; percent[b] = outliers / (sum(valid)[b] + 1e-9) (loss/flow.py:609-649). */
typedef struct snnflow_aee_args {
    int B, H, W;
    const float* flow;          /* [B][2][H][W] network flow (before scaling) */
    const float* gtflow;        /* [B][2][H][W] */
    const float* event_mask;    /* [B][H][W] event mask of the last window */
    const float* dt_ratio;      /* [B] dt_gt / dt_input, or NULL: the ratio of dt_gt / dt_input below */
    float flow_scaling;
    double* acc;                /* ABI 29: scratch of snnflow_aee_acc_doubles(B, H, W) doubles; acc[0] (a
                                 * completion counter) must be zero before the first call on it and every
                                 * call leaves it zero -- allocate zeroed once and reuse */
    float* aee; float* percent; /* out [B] */
    /* ABI 31 (dt_ratio NULL): dt_gt[b] / dt_input[b] formed in the kernel, each of dt_gt_n / dt_input_n
     * (1: one value for the batch, or B) entries -- no separate division launch per window */
    const float* dt_gt; const float* dt_input; int dt_gt_n, dt_input_n;
} snnflow_aee_args;
/* One launch: per-block partial sums (fp64 rows), the last block to finish reduces them in a fixed
 * order (deterministic) and writes aee / percent.  The scratch carries the completion counter from
 * call to call: one stream at a time per scratch (concurrent calls need their own scratch). */
int snnflow_aee(const snnflow_aee_args* a, void* stream);
int snnflow_aee_acc_doubles(int B, int H, int W);

/* Every flow-vs-ground-truth metric of loss/flow.py in one pass over the pixels
 * (flow' = flow*flow_scaling*dt_ratio[b], valid = event_mask && gt != (0,0)):
 *   out[b][SNNFLOW_M_AEE], [_AEE_PCT]   AEE (:597-649): same as snnflow_aee
 *   [_NEE], [_NEE_PCT]    NEE (:651-701): |f'-g| / (min(|f'|,|g|) + 0.01); outliers
 *                         (masked error > 0.5) counted over the whole batch
 *   [_AAE], [_AAE_PCT]    AAE (:703-762): acos(clamp((|f'||g|) / (f'.g + 0.01))) (the
 *                         reference's formula); outliers (> pi/6) per sample
 *   [_NAAE]               NAAE (:764-820): acos(clamp(f'.g / (|f'||g| + 1e-9))) / (|f'| + 1e-9)
 *   [_AE_OF_MEANS]        AE_ofMeans (:822-883): angle between the masked means
 *   [_AAE_WEIGHTED]       AAE_Weighted (:885-909): sum(ang*|f'|) over ALL pixels /
 *                         (sum(|f'|*valid) + 1e-9) (the reference does not mask the numerator)
 *   [_AAE_FILTERED]       AAE_Filtered (:911-937): mean ang over valid && |f'| >= mag_threshold
 * Per-pixel terms are reduced per block into rows (scratch snnflow_flow_metrics_rows
 * doubles) and summed in a fixed order: deterministic. */
#define SNNFLOW_M_AEE 0
#define SNNFLOW_M_AEE_PCT 1
#define SNNFLOW_M_NEE 2
#define SNNFLOW_M_NEE_PCT 3
#define SNNFLOW_M_AAE 4
#define SNNFLOW_M_AAE_PCT 5
#define SNNFLOW_M_NAAE 6
#define SNNFLOW_M_AE_OF_MEANS 7
#define SNNFLOW_M_AAE_WEIGHTED 8
#define SNNFLOW_M_AAE_FILTERED 9
#define SNNFLOW_NUM_METRICS 10
typedef struct snnflow_flow_metrics_args {
    int B, H, W;
    const float* flow; const float* gtflow; const float* event_mask; const float* dt_ratio;
    float flow_scaling, mag_threshold;
    double* rows;               /* scratch snnflow_flow_metrics_rows(B, H, W) doubles */
    float* out;                 /* out [B][SNNFLOW_NUM_METRICS] */
} snnflow_flow_metrics_args;
int snnflow_flow_metrics(const snnflow_flow_metrics_args* a, void* stream);
int snnflow_flow_metrics_rows(int B, int H, int W);

/* HIP twin of the export op SNN_implementation::LIF (ONNX_LIF_operator/src/lif_op.cpp:8-56):
 * m' = beta[c]*mem + x; spk = m' >= thr[c]; mem_out = spk ? 0 : m'  (NCHW). */
int snnflow_lif_export(const float* x, const float* mem, const float* beta, const float* thr,
                       int N, int C, int HW, float* spk, float* mem_out, void* stream);

/* Threshold gradient of the subtract-reset neuron (snn.Leaky reset_mechanism "subtract",
 * SNNtorch_spiking_submodules.py:171, hard_reset=False): v = beta*m + I - r*theta with the reset
 * r = H(m - theta) detached, so theta also receives -sum r * dL/dv through v; the fused LIF
 * backward kernels form the zero-reset part -sum dL/dv.  Adds -sum_px [mem - thr > 0] * g_cur
 * per channel to g_theta[c] (g_cur = dL/dv and mem = the incoming membrane, NHWC [npix][c]).
 * Deterministic: per-block channel totals go to scratch (SNNFLOW_THETA_SCRATCH floats) and one
 * block sums them in block order (fp64).  c = 4, 8, 16 or 32. */
#define SNNFLOW_THETA_BLOCKS 1024
#define SNNFLOW_THETA_SCRATCH (SNNFLOW_THETA_BLOCKS * 32)
int snnflow_lif_theta_subtract(const float* g_cur, const float* mem, const float* thr, int64_t npix, int c,
                               float* g_theta, float* scratch, void* stream);

/* clip_grad_norm_ (train_flow.py:265-266) over one flat gradient buffer of n floats, in place:
 * total = ||g||_2, g *= min(max_norm / (total + eps), 1); total_out (device, may be NULL). */
int snnflow_clip_grad_norm(float* g, int64_t n, float max_norm, float eps, float* total_out, void* stream);
/* The same for large vectors (grid-wide, 3 launches, deterministic fixed-order fp64 partials);
 * scratch: SNNFLOW_CLIP_SCRATCH doubles. */
#define SNNFLOW_CLIP_SCRATCH 513
int snnflow_clip_grad_norm_large(float* g, int64_t n, float max_norm, float eps, float* total_out,
                                 double* scratch, void* stream);

/* ---- evaluation forward (eval_flow.py:208-338: model.eval(), BatchNorm on running statistics)
 * One layer-step with conv + BatchNorm + LIF fused, and for the last layer also the prediction
 * ConvLayer(C->2, 1x1) + tanh (models/model.py:182): with running statistics a layer's spikes can
 * leave the kernel that computes its conv, so task (l, t) reads the spikes of layer l-1 at step t
 * (or the event tensor, l = 0) and layer l's own state at t-1, and writes layer l's state at t.  The
 * T x L layer-steps then run in T + L - 1 wavefront launches (task (l, t) in launch l + t) instead of
 * the train path's 2(T-1) + L + 1 split conv / LIF launches.  c = 8; the same per-element LIF
 * arithmetic as the train-path kernels (snnflow_lif_fwd / the LIF-fed conv tasks). */
typedef struct snnflow_eval_fwd_args {
    int B, H, W, cin, c;
    const float* x; int64_t xs_b, xs_c, xs_h, xs_w;  /* cin != c (2 or 4): the event tensor, any strides */
    const float* s_in;        /* cin == c: spikes of layer l-1 at this step, NHWC [B][H][W][c] (its state's
                               * spike half) */
    const float* mem_prev;    /* NHWC [B][H][W][c] membrane of this layer at t-1 (NULL: zero) */
    const float* s_prev;      /* recurrent cells: NHWC spikes of this layer at t-1 (NULL: no recurrent input) */
    const float* wt_ff; const float* wt_rec;      /* [tap][cin][c] (snnflow_prep_desc.wt_fwd) */
    const float* wt_ff_t; const float* wt_rec_t;  /* [tap][c][cin] (wt_bwd): the c = 8 matrix-core fragments */
    snnflow_neuron n;         /* this layer's BatchNorm (bn_train must be 0) + LIF */
    float* state;             /* out [2][B][H][W][c]: membrane, spikes */
    const float* pred_w; const float* pred_b; float* flow;  /* optional (last layer): flow [B][2][H][W] */
} snnflow_eval_fwd_args;
#define SNNFLOW_EVAL_MAX_TASKS 8
int snnflow_eval_slot(const snnflow_eval_fwd_args* tasks, int n, void* stream);

/* clip_grad_norm_ + Adam in one launch (train_flow.py:265-267: clip_grad_norm_(params, max_norm),
 * optimizer.step() of torch.optim.Adam, configs/train_SNN.yml:45-47), over the engine's flat gradient
 * buffer (snnflow.optim.ClipAdam).  total = ||grad||_2 (fp64), grad *= min(max_norm / (total +
 * clip_eps), 1) in place (skipped when max_norm <= 0), *step += 1, then per element the reference's
 * Adam (torch _single_tensor_adam: weight decay, exp_avg.lerp_(g, 1 - beta1), exp_avg_sq =
 * exp_avg_sq * beta2 + (1 - beta2) g^2, bias corrections in fp64, denom = sqrt(exp_avg_sq) /
 * sqrt(bc2) + eps, param -= lr / bc1 * exp_avg / denom).  t[i] maps parameter tensor i to
 * grad[offset .. offset + numel) and to exp_avg / exp_avg_sq[state_offset .. state_offset + numel)
 * (persistent moment buffers: the gradient buffer may move between steps, the moments do not); the
 * t[] in ascending, non-overlapping gradient order.  n <= SNNFLOW_CLIP_ADAM_MAX_N; up to
 * SNNFLOW_CLIP_ADAM_ONE_BLOCK elements one launch of one block, above that (ABI 32) two launches of
 * one block per SNNFLOW_CLIP_ADAM_ONE_BLOCK elements (per-block norm partials in `scratch`,
 * SNNFLOW_CLIP_SCRATCH doubles, summed by every block in the same order: deterministic).  Replaces snnflow_clip_grad_norm + torch's Adam kernels. */
#define SNNFLOW_ADAM_MAX_TENSORS 64
#define SNNFLOW_CLIP_ADAM_MAX_N (1 << 20)
#define SNNFLOW_CLIP_ADAM_ONE_BLOCK 8192
typedef struct {
    float* param;
    int64_t offset;        /* into grad */
    int64_t state_offset;  /* into exp_avg / exp_avg_sq */
    int64_t numel;
} snnflow_adam_tensor;
typedef struct {
    float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    float* step;       /* device scalar (fp32, as torch's capturable Adam state) */
    float* total_out;  /* device scalar or NULL: the pre-clip norm */
    int64_t n;
    double lr, beta1, beta2, eps, weight_decay;
    float max_norm, clip_eps;
    int ntensors;
    snnflow_adam_tensor t[SNNFLOW_ADAM_MAX_TENSORS];
    double* scratch;   /* ABI 32: SNNFLOW_CLIP_SCRATCH doubles when n > SNNFLOW_CLIP_ADAM_ONE_BLOCK (else may be NULL) */
} snnflow_clip_adam_args;
int snnflow_clip_adam(const snnflow_clip_adam_args* a, void* stream);

/* Activity log of LIFFireNet.forward(log=True) (models/model.py:188-205: per tensor
 * `l.detach().ne(0).float().mean()`): counts[i] = number of non-zero elements (NaN counts, -0 does
 * not) of the i-th dense fp32 region ptrs[i][0 .. sizes[i]).  ptrs/sizes are host arrays of n <=
 * SNNFLOW_MAX_COUNT_TENSORS entries; counts is a device array of n uint64, overwritten.  Exact
 * integer counts (wavefront ballots + popcount, integer atomics): order-independent. */
#define SNNFLOW_MAX_COUNT_TENSORS 16
int snnflow_count_nonzero(const float* const* ptrs, const int64_t* sizes, int n, uint64_t* counts, void* stream);

/* ---- Spiking U-Net: SpikingRecEVFlowNet (models/model.py:723-858) =
 *      SpikingMultiResUNetRecurrent (models/unet.py:414-461) of ConvLIF / ConvLIFRecurrent cells
 *      (models/spiking_submodules.py:29-300) in SpikingRecurrentConvLayer (:303-346),
 *      SpikingResidualBlock (:349-385) and SpikingUpsampleConvLayer (:388-417) blocks.
 *
 * Every convolution is an implicit GEMM on the bf16 matrix cores (v_mfma_f32_16x16x32_bf16):
 * D[m][pixel] = sum_k A[m][k] * X[k][pixel].  The pixel operand X is a bf16 NHWC "act" tensor
 * whose values are exact in bf16 (spikes 0/1, residual sums 0..3, their bilinear upsamples k/16,
 * and fp32 values pre-split into hi/mid/lo bf16 channels); the weight operand is stored split
 * into three bf16 parts (hi, mid, lo), so every product is the exact fp32 product and the
 * accumulation is fp32.  Act tensors: [B][H][W][cpitch] bf16 (uint16_t here), cpitch % 32 == 0,
 * padding channels zero.  "k positions" = the act's channels; a kmap (int [cpitch]) names the
 * reference input channel of each position (-1: padding), so one weight tensor of the reference
 * feeds several positions (hi/mid/lo splits of an fp32 channel). */
#define SNNFLOW_UNET_MAX_SEGS 4
#define SNNFLOW_UNET_MODE_S1 0   /* stride-1 conv, pad ksize/2 */
#define SNNFLOW_UNET_MODE_S2 1   /* stride-2 conv, pad ksize/2 */
#define SNNFLOW_UNET_MODE_T2 2   /* transposed stride-2 conv (input gradient of a MODE_S2 conv) */
#define SNNFLOW_UNET_EPI_STORE 0 /* out[pix*ld + m] = (or +=) D */
#define SNNFLOW_UNET_EPI_LIF 1   /* ConvLIF membrane / spike / state epilogue (spiking_submodules.py:121-151, 265-300) */
#define SNNFLOW_SG_ARCTAN 0      /* spiking_util.py:82-93, 108-109 */
#define SNNFLOW_SG_SUPERSPIKE 1  /* :28-43, 96-97 */
#define SNNFLOW_SG_MGSPIKE 2     /* :46-65, 100-101 */
#define SNNFLOW_SG_TRIANGLE 3    /* :68-79, 104-105 */

typedef struct {
    const uint16_t* x;  /* act tensor bf16 [B][H][W][cpitch] */
    int H, W, cpitch;
    int mode;           /* SNNFLOW_UNET_MODE_* */
    int kc0;            /* first 32-channel weight chunk of this segment within a tap */
    int nparts;         /* weight parts multiplied with it: 3 (exact operand); 2, 1 for the mid / lo
                           planes of a split operand (drops products below 2^-24 relative) */
} snnflow_unet_seg;

typedef struct {
    int B, Ho, Wo;      /* output pixels: GEMM N = B*Ho*Wo */
    int M;              /* valid output channels (GEMM M) */
    int ksize;          /* odd conv kernel size (3) */
    int nseg;
    snnflow_unet_seg seg[SNNFLOW_UNET_MAX_SEGS];
    const uint16_t* w;  /* bf16 [3][ksize^2][kct][mpad][32] (snnflow_unet_prep_weights) */
    int kct, mpad;
    int xparts;         /* 1: segments exact in bf16; 3: every segment is an fp32 tensor split into hi / mid /
                           lo bf16 planes xpart elements apart (the 6 products above 2^-24 relative) */
    int64_t xpart;
    int pclass;         /* -1: all output pixels; 0..3: the parity class (py = pclass >> 1, px = pclass & 1) of
                           a single MODE_T2 segment, whose taps of the other parities are skipped */
    int epi;            /* SNNFLOW_UNET_EPI_* */
    /* EPI_STORE */
    float* out; int ld; int accumulate;
    /* EPI_LIF (ConvLIF cell; M = hidden channels, output resolution = cell resolution) */
    const float* leak; const float* thresh; int hard_reset;
    const float* prev_state;   /* fp32 [2][B][Ho][Wo][M] (v, z) or NULL (zeros) */
    const uint16_t* residual;  /* act [pix][res_pitch] added to the spikes, or NULL */
    int res_pitch;
    float* state;              /* fp32 [2][B][Ho][Wo][M] out (v_out, z_out) */
    float* current;            /* fp32 [pix][M] out: ff (+ rec), for the backward */
    uint16_t* act;             /* act [pix][act_pitch] out: z_out (+ residual) */
    int act_pitch;
    /* ABI 18, split-K (ksplit 0 or 1: off): the k-steps of every output tile are dealt to ksplit blocks,
     * each writing its fp32 partial tile to partial [ksplit][P][M] (P = output pixels of the launch's
     * domain); a second kernel sums them in split order (deterministic) and applies the epilogue.  For
     * the deep layers, whose output tiles alone leave most of the 256 CUs idle. */
    int ksplit;
    float* partial;
} snnflow_unet_conv_args;
#define SNNFLOW_UNET_MAX_KSPLIT 16
/* Split-K factor the library chooses for a launch (1: none); the caller then sets ksplit and a
 * partial buffer of ksplit * P * M floats. */
int snnflow_unet_conv_ksplit(const snnflow_unet_conv_args* a);

/* Convolution (forward of a cell with the LIF epilogue, or an input gradient with EPI_STORE). */
int snnflow_unet_conv(const snnflow_unet_conv_args* a, void* stream);

/* Weight operand of snnflow_unet_conv from a torch conv weight w [cout][cin][k][k] (fp32):
 * forward (transpose 0): dst[p][tap][kc0 + kc][m][kk] = part p of w[m][kmap[32 kc + kk]][tap]
 *   for kc < nkc (m < cout; kmap entry -1 or m >= cout: 0);
 * input gradient (transpose 1): dst[p][tap'][kc][m][kk] = part p of w[32 kc + kk][kmap[m]][tap],
 *   m < mvalid (the gradient's k positions), tap = flip ? k^2-1-tap' : tap'.  dst is not cleared:
 *   the caller zero-fills once (padding entries are never written). */
int snnflow_unet_prep_weights(const float* w, int cout, int cin, int ksize, const int* kmap, int transpose,
                              int flip, int mvalid, int kc0, int nkc, int kct, int mpad, uint16_t* dst,
                              void* stream);

/* Weight gradient of one input segment, accumulated (fp32 atomics) over pixels and calls:
 * dwk[tap][k0 + k][m] += sum_pix X[gather(pix, tap)][k] * G[pix][m], G = g3 hi + mid + lo planes
 * ([3][B*Ho*Wo][gpitch] bf16, part stride gpart), k < seg.cpitch. */
typedef struct {
    int B, Ho, Wo, M, ksize;
    const uint16_t* g3; int gpitch; int64_t gpart;
    snnflow_unet_seg seg;
    int k0, ktot;       /* first k position of the segment in dwk, k positions per tap in dwk */
    float* dwk;         /* fp32 [ksize^2][ktot][M] */
    /* ABI 19, optional: workspace of snnflow_unet_wgrad_partial_floats() floats; with it the pixel
     * splits write partial tiles that one more kernel adds to dwk in split order (deterministic, no
     * atomics); NULL: fp32 atomics into dwk */
    float* partial;
} snnflow_unet_wgrad_args;
int64_t snnflow_unet_wgrad_partial_floats(const snnflow_unet_wgrad_args* a);
int snnflow_unet_wgrad(const snnflow_unet_wgrad_args* a, void* stream);

/* dw[m][c][tap] (+)= sum over the (up to 3) positions k of input channel c (kmap_inv [cin][3], -1:
 * none; positions relative to k0) of dwk[tap][k0 + k][m] (torch layout [cout][cin][k][k]). */
int snnflow_unet_wgrad_finalize(const float* dwk, int ktot, const int* kmap_inv, int k0, int nk, int cout, int cin,
                                int ksize, int accumulate, float* dw, void* stream);

/* ConvLIF backward of one cell and step, per element (spiking_submodules.py:121-151, 265-300):
 * x = v_out - th, sg = surrogate(x, width), gxs = (g_out + g_z) * sg, gv = g_v + gxs (+ residual
 * path), g_cur = gv * (1 - leak) written as hi/mid/lo bf16 planes (padding channels 0);
 * g_prev v-half = gv*leak*(1-z) (hard) | gv*leak (soft); z-half = 0 (detach) or the reset term;
 * g_res += g_out; sums of dL/dthresh and dL/dleak(before sigmoid') into acc (fp64 [2*C]). */
typedef struct {
    int P, C;
    const float* leak; const float* thresh; float width; int hard_reset, detach, surrogate;
    const float* g_out; int g_pitch;           /* fp32 [P][g_pitch] or NULL */
    const float* g_state;                       /* fp32 [2][P][C] or NULL */
    const float* state; const float* prev_state; const float* current;
    uint16_t* g_cur3; int gc_pitch; int64_t gc_part;
    float* g_prev;                              /* fp32 [2][P][C] or NULL */
    float* g_res; int gres_pitch;               /* or NULL */
    double* acc;                                /* [2*C] */
    /* ABI 25, optional: workspace of snnflow_unet_lif_bwd_partial_doubles(P, C, gc_pitch) doubles ([2C][blocks]); with
     * it every block writes its sums there and a second kernel adds them to acc in block order
     * (deterministic, and no contention of ~2,000 blocks' fp64 atomics on 2*C addresses); NULL: the
     * blocks add to acc by fp64 atomics. */
    double* partial;
    /* ABI 26: 1 = g_res is written (g_res = g_out: its first contribution), 0 = added to. */
    int res_assign;
} snnflow_unet_lif_bwd_args;
int snnflow_unet_lif_bwd(const snnflow_unet_lif_bwd_args* a, void* stream);
int snnflow_unet_lif_bwd_partial_doubles(int P, int C, int gc_pitch);

/* g_thresh = (thresh >= 0.01) * acc[c], g_leak = acc[C + c] * s * (1 - s), s = sigmoid(leak). */
int snnflow_unet_cell_param_grads(const double* acc, const float* leak, const float* thresh, int C, int accumulate,
                                  float* g_leak, float* g_thresh, void* stream);

/* fp32 channels (strided, e.g. NCHW or a state half) -> act [P][cpitch] bf16 with channels
 * [hi(C) | mid(C) | lo(C) | 0] (split 1), or [value(C) | 0] (split 0, values exact in bf16). */
int snnflow_unet_pack(const float* src, int B, int H, int W, int C, int64_t sb, int64_t sc, int64_t sh,
                      int64_t sw, int split, uint16_t* dst, int cpitch, void* stream);

/* Decoder input (unet.py:455-458 + spiking_submodules.py:415): bilinear x2 upsample
 * (align_corners=False) of cat(pred, x, block) at h x w into act [B][2h][2w][cpitch] with
 * channels [x (cx) | block (cb) | pred hi0 hi1 mid0 mid1 lo0 lo1 (if pred) | 0]. */
int snnflow_unet_dec_in(const uint16_t* x, int cx, int px, const uint16_t* block, int cb, int pb,
                        const float* pred, int B, int h, int w, uint16_t* dst, int cpitch, void* stream);
/* Its backward from g_up fp32 [B][2h][2w][gpitch]: g_x [pix][gx_pitch] +=, g_block +=,
 * g_pred [B][2][h][w] = (the pred channels' gradient at its hi position).  assign (ABI 26): bit 0
 * writes g_x, bit 1 writes g_block (=, their first contribution; else +=). */
int snnflow_unet_dec_in_bwd(const float* g_up, int gpitch, int cx, int cb, int has_pred, int B, int h, int w,
                            float* g_x, int gx_pitch, float* g_block, int gb_pitch, float* g_pred, int assign,
                            void* stream);

/* Prediction layer (submodules.py:96-113, 1x1 conv + bias + tanh, unet.py:351-365) and the
 * nearest upsample to the input resolution (model.py:840-850):
 * flow = tanh(W x + b) [B][2][h][w]; flow_full [B][2][h*s][w*s] (s = up). */
int snnflow_unet_pred_fwd(const uint16_t* x, int cpitch, int C, const float* w, const float* b, int B, int h,
                          int wd, int up, float* flow, float* flow_full, void* stream);
/* g_pre = (1 - flow^2) * (sum of g_full over the s x s block + g_extra) into gpre [B][2][h][w];
 * g_x[pix][gx_pitch] += W^T g_pre (assign, ABI 26: = instead of +=); acc (fp64 [2C + 2]) += (dW, db)
 * sums.  partial (ABI 26, optional): workspace of snnflow_unet_pred_bwd_partial_doubles doubles; with
 * it the blocks' sums are added to acc in a fixed order (bit-reproducible), else by fp64 atomics. */
int snnflow_unet_pred_bwd(const uint16_t* x, int cpitch, int C, const float* w, const float* flow,
                          const float* g_full, const float* g_extra, int B, int h, int wd, int up, float* gpre,
                          float* g_x, int gx_pitch, double* acc, int assign, double* partial, void* stream);
int snnflow_unet_pred_bwd_partial_doubles(int B, int h, int wd, int C);
int snnflow_unet_pred_param_grads(const double* acc, int C, int accumulate, float* g_w, float* g_b, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Per-time-step driver of the LIFFireNet family (csrc/firenet_step.cpp, host code): one call
 * launches the L+1 forward kernels of a time step (snnflow_conv_fwd x L + snnflow_lif_fwd), one
 * call the L+1 backward kernels (snnflow_lif_bwd + snnflow_layer_bwd x L), one call the deferred
 * weight gradients of a BPTT window (snnflow_wgrad per layer + snnflow_slab_reduce).  It replaces
 * the Python argument building of the eager drop-in path (models/model.py:135-207 called once
 * per window by train_flow.py:231-279); the kernels and their arguments are those of the
 * single-kernel entry points above.  The plan holds what is constant across steps; the io
 * structs what each step allocates.
 * ------------------------------------------------------------------------------------------- */
typedef struct snnflow_firenet_plan {
    int L, B, H, W, c, cin0;
    int rec[SNNFLOW_MAX_LAYERS];
    int train[SNNFLOW_MAX_LAYERS];          /* BatchNorm batch statistics (else running) */
    snnflow_neuron n[SNNFLOW_MAX_LAYERS];
    const float* wt_fwd_ff[SNNFLOW_MAX_LAYERS];
    const float* wt_fwd_rec[SNNFLOW_MAX_LAYERS];
    const float* wt_bwd_ff[SNNFLOW_MAX_LAYERS];
    const float* wt_bwd_rec[SNNFLOW_MAX_LAYERS];
    const uint16_t* wf_ff[SNNFLOW_MAX_LAYERS];   /* forward fragments (c = 16, 32) or NULL */
    const uint16_t* wf_rec[SNNFLOW_MAX_LAYERS];
    const uint16_t* wd_ff[SNNFLOW_MAX_LAYERS];   /* input-gradient fragments or NULL */
    const uint16_t* wd_rec[SNNFLOW_MAX_LAYERS];
    double* fwd_acc; int64_t fwd_acc_stride;     /* [L][stride] doubles, zero_n = stride */
    double* bwd_acc; int64_t bwd_acc_stride;
    const float* pred_w; const float* pred_b;
    float* slab_ff[SNNFLOW_MAX_LAYERS];          /* per-block weight-gradient slabs */
    float* slab_rec[SNNFLOW_MAX_LAYERS];
    int nblk;
} snnflow_firenet_plan;

typedef struct snnflow_firenet_fwd_io {
    const float* x; int64_t xs[4];               /* event tensor (strided b, c, h, w) */
    float* ys;                                   /* [L][B][H][W][c] pre-BN currents */
    float* stats;                                /* [L][2][c] */
    float* states;                               /* [L][2][B][H][W][c] */
    float* flow;                                 /* [B][2][H][W] */
    const float* mem_in[SNNFLOW_MAX_LAYERS];     /* incoming membranes (NHWC) or NULL (zeros) */
    const float* s_prev[SNNFLOW_MAX_LAYERS];     /* previous spikes of recurrent layers or NULL */
} snnflow_firenet_fwd_io;
int snnflow_firenet_fwd(const snnflow_firenet_plan* p, const snnflow_firenet_fwd_io* io, void* stream);

typedef struct snnflow_firenet_bwd_io {
    const float* ys; const float* stats; const float* flow;
    const float* mem_in[SNNFLOW_MAX_LAYERS];
    const float* g_state[SNNFLOW_MAX_LAYERS];    /* grads of the state outputs (NHWC states) or NULL */
    const float* g_flow; int64_t gflow_sb, gflow_sc;
    float* g_cur;                                /* [L][B][H][W][c] out */
    float* bnc;                                  /* [L][2][c] out */
    float* g_prev[SNNFLOW_MAX_LAYERS];           /* grads of the previous states or NULL */
    int ext[SNNFLOW_MAX_LAYERS];                 /* previous state not produced by this model */
    float* g_x; int64_t gxs[4];                  /* head input gradient or NULL */
    snnflow_neuron_grad ng[SNNFLOW_MAX_LAYERS];
    float* g_pred_w; float* g_pred_b;
    int accumulate;                              /* add into the neuron / pred gradients */
} snnflow_firenet_bwd_io;
int snnflow_firenet_bwd(const snnflow_firenet_plan* p, const snnflow_firenet_bwd_io* io, void* stream);

/* ABI 37: the backwards of T consecutive time steps of one BPTT chain in wavefront launches
 * (snnflow_bwd_slot: task (kernel j, reversed step tau) in launch j + 2 tau, as engine.FireNetSequence),
 * for the per-window drop-in loop whose T model() calls are T autograd nodes: the chain's first step
 * (the last node autograd calls) issues every step's backward in one call.  Steps in time order; each
 * step t's tensors as snnflow_firenet_fwd wrote them (ys, stats, flow, states [L][2][B][H][W][c]); its
 * incoming states are step t-1's (step 0: mem_in0 / s_prev0).  Gradients: g_flow[t] (NULL: none) with
 * element strides (batch, channel); g_state_last = dL/d(the last step's output states) or NULL;
 * inside the chain the spike halves of the recurrent layers' state gradients live in g_out ((T-1) x
 * (recurrent layers) buffers of 2BHWc floats, step-major, layer order; the membrane half is never
 * read); g_prev0[l]: dL/d(step 0's incoming state l) (written when non-NULL: spike half for a recurrent
 * layer, plus the zero-filled / ext0 membrane half).  g_cur / bnc: [T][L] x the per-step outputs of
 * snnflow_firenet_bwd.  bwd_acc: T*L backward accumulators (step-major, acc_stride doubles apart,
 * SNNFLOW_ACC_LEN(SNNFLOW_BWD_ACC(c)) each), zero on entry.  fresh = 1: the first task of every
 * layer writes (does not add to) the neuron / pred gradients.  fused = 1 (c = 8): the weight
 * gradients of layers >= 1 go into plan->slab_* inside the backward tasks, slab_live[l] in/out (0: the
 * layer's slab rows are written, 1: added to); layer 0's (and, with fused = 0, every layer's) stay for
 * snnflow_firenet_wgrad.  c = 8, 16 or 32 (snnflow_slot_supported); 1 <= T <= SNNFLOW_MAX_WINDOWS. */
typedef struct snnflow_firenet_seq_bwd {
    int T, fresh, fused;
    const float* ys[SNNFLOW_MAX_WINDOWS];
    const float* stats[SNNFLOW_MAX_WINDOWS];
    const float* flow[SNNFLOW_MAX_WINDOWS];
    const float* states[SNNFLOW_MAX_WINDOWS];
    const float* g_flow[SNNFLOW_MAX_WINDOWS];
    int64_t gflow_sb[SNNFLOW_MAX_WINDOWS], gflow_sc[SNNFLOW_MAX_WINDOWS];
    const float* mem_in0[SNNFLOW_MAX_LAYERS];
    const float* s_prev0[SNNFLOW_MAX_LAYERS];
    float* g_prev0[SNNFLOW_MAX_LAYERS];
    int ext0[SNNFLOW_MAX_LAYERS];
    const float* g_state_last[SNNFLOW_MAX_LAYERS];
    float* g_out;
    float* g_cur; float* bnc;
    double* bwd_acc; int64_t acc_stride;
    snnflow_neuron_grad ng[SNNFLOW_MAX_LAYERS];
    float* g_pred_w; float* g_pred_b;
    /* ABI 40: fuse_head = 1 adds the head's weight gradient of every step to the plan's slab_ff[0] rows
     * inside the head's backward tasks (layer 0 feed-forward, cin0 2 or 4), reading the step inputs
     * x[t] (strides xs[t] = b, c, h, w); the caller then leaves layer 0 out of the deferred weight
     * gradients.  slab_live[0] is read and set like the fused layers'. */
    int fuse_head;
    const float* x[SNNFLOW_MAX_WINDOWS];
    int64_t xs[SNNFLOW_MAX_WINDOWS][4];
} snnflow_firenet_seq_bwd;
int snnflow_firenet_bwd_seq(const snnflow_firenet_plan* p, const snnflow_firenet_seq_bwd* q, int* slab_live,
                            void* stream);

/* One time step's tensors for the deferred weight gradients (the backward's g_cur / bnc and the
 * forward's ys / stats / states, the step's input and the previous spikes). */
typedef struct snnflow_firenet_wgrad_step {
    const float* g_cur; const float* bnc; const float* ys; const float* stats;
    const float* x; int64_t xs[4];
    const float* states;
    const float* s_prev[SNNFLOW_MAX_LAYERS];
} snnflow_firenet_wgrad_step;
/* Weight gradients of every layer over nsteps steps (order as given) into the plan's slabs, then
 * the fixed-order slab sums into g_ff[l] / g_rec[l]. */
int snnflow_firenet_wgrad(const snnflow_firenet_plan* p, const snnflow_firenet_wgrad_step* steps, int nsteps,
                          float* const* g_ff, float* const* g_rec, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Standalone BatchNorm2d over [P][C] channel-fastest rows (csrc/norm.hip): MPBN of the membrane
 * (SNNtorch_spiking_submodules.py:66-121, applied at :313-317 / :558-562) and TEBN's inner BN
 * (:18-63) when called as modules.  C must divide 256.  Train: fp64 batch sums (fixed-order
 * partials), biased variance to normalise, unbiased variance into running_var with momentum,
 * num_batches_tracked += 1; eval: running statistics.  save_mean / save_invstd [C] are written in
 * both modes (the backward's inputs).  scratch: snnflow_bn_scratch_doubles(C) doubles.
 * ------------------------------------------------------------------------------------------- */
#define SNNFLOW_BN_PARTS 256
typedef struct {
    int64_t P;
    int C;
    int train;
    const float* x;
    float* y;
    const float* weight;  /* [C] or NULL (affine off) */
    const float* bias;    /* [C] or NULL */
    float* running_mean;  /* [C] or NULL (track_running_stats=False; train only) */
    float* running_var;
    int64_t* num_batches_tracked; /* or NULL */
    float momentum, eps;
    float* save_mean;
    float* save_invstd;
    double* scratch;
} snnflow_bn_fwd_args;
int snnflow_bn_fwd(const snnflow_bn_fwd_args* a, void* stream);

/* g_weight = sum g*xhat, g_bias = sum g (either NULL to skip); g_x (or NULL) = the BatchNorm input
 * gradient (train: through the batch statistics; eval: weight*invstd*g). */
typedef struct {
    int64_t P;
    int C;
    int train;
    const float* x;
    const float* g;
    const float* weight;
    const float* save_mean;
    const float* save_invstd;
    float* g_x;
    float* g_weight;
    float* g_bias;
    double* scratch;
} snnflow_bn_bwd_args;
int snnflow_bn_bwd(const snnflow_bn_bwd_args* a, void* stream);
int snnflow_bn_scratch_doubles(int C);

/* ConvLayer with a 1x1 kernel (models/submodules.py:16-113; LIFFireNet's pred, model.py:105-107,
 * the U-Net's multires preds, unet.py:255-262, cin up to 8 x base channels; called as a module):
 * out [B][cout][H][W] = act(W x + b), x of any strides (elements, b c h w).
 * Backward: g_pre = g_out * act'(out) (from the output), g_x (if set, strides gxs) = W^T g_pre,
 * g_w [cout][cin] / g_b [cout] (either NULL to skip) as fixed-order fp64 sums;
 * scratch: SNNFLOW_BN_PARTS * cout * (cin + 1) doubles. */
#define SNNFLOW_ACT_NONE 0
#define SNNFLOW_ACT_TANH 1
#define SNNFLOW_ACT_RELU 2
#define SNNFLOW_ACT_SIGMOID 3
#define SNNFLOW_PW_MAX_CIN 256
#define SNNFLOW_PW_MAX_COUT 4
typedef struct {
    int B, H, W, cin, cout, act;
    const float* x;
    int64_t xs[4];
    const float* w;
    const float* b;
    float* out;
    float* g_x;
    int64_t gxs[4];
} snnflow_pointwise_args;
int snnflow_pointwise_fwd(const snnflow_pointwise_args* a, void* stream);
int snnflow_pointwise_bwd(const snnflow_pointwise_args* a, const float* g_out, int64_t gs_b, int64_t gs_c,
                          float* g_w, float* g_b, double* scratch, void* stream);

const char* snnflow_last_error(void);
int snnflow_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
