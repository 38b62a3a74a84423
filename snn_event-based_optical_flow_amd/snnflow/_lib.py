"""ctypes binding of the snnflow C-ABI (include/snnflow.h).

The HIP library is the product: there is no CPU fallback.  Importing this module
fails loudly when libsnnflow.so is missing; calls fail loudly when there is no GPU.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SNNFLOW_LIB", os.path.join(_HERE, "libsnnflow.so"))

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_int64
F32 = ctypes.c_float
F64 = ctypes.c_double

TILE_H, TILE_W = 8, 32
ABI_VERSION = 40
THETA_SCRATCH = 1024 * 32  # SNNFLOW_THETA_SCRATCH


class Neuron(ctypes.Structure):
    _fields_ = [("bn_weight", P), ("bn_bias", P), ("running_mean", P), ("running_var", P),
                ("num_batches_tracked", P), ("beta", P), ("threshold", P),
                ("momentum", F64), ("eps", F64), ("bn_train", I32), ("zero_reset", I32)]


class NeuronGrad(ctypes.Structure):
    _fields_ = [("bn_weight", P), ("bn_bias", P), ("beta", P), ("threshold", P)]


class ConvFwdArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("cin", I32), ("c", I32), ("lif_in", I32),
                ("x", P), ("xs_b", I64), ("xs_c", I64), ("xs_h", I64), ("xs_w", I64),
                ("prev_y", P), ("prev_mem", P), ("prev_acc", P), ("prev_stats", P),
                ("prev", Neuron), ("prev_state", P),
                ("wt_ff", P), ("wt_rec", P), ("wt_ff_t", P), ("wt_rec_t", P), ("s_prev", P),
                ("y", P), ("acc", P), ("zero0", P), ("zero1", P), ("zero_n", I32),
                ("wf_ff", P), ("wf_rec", P), ("state_spk_skip", I32), ("prev_spk_bits", P), ("s_prev_bits", P)]


class EvalFwdArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("cin", I32), ("c", I32),
                ("x", P), ("xs_b", I64), ("xs_c", I64), ("xs_h", I64), ("xs_w", I64),
                ("s_in", P), ("mem_prev", P), ("s_prev", P), ("wt_ff", P), ("wt_rec", P), ("wt_ff_t", P),
                ("wt_rec_t", P), ("n", Neuron), ("state", P), ("pred_w", P), ("pred_b", P), ("flow", P)]


EVAL_MAX_TASKS = 8  # SNNFLOW_EVAL_MAX_TASKS


class LifFwdArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("c", I32),
                ("y", P), ("mem", P), ("acc", P), ("stats", P), ("n", Neuron), ("state", P),
                ("pred_w", P), ("pred_b", P), ("flow", P),
                ("zero0", P), ("zero1", P), ("zero_n", I32), ("state_spk_skip", I32)]


class LifBwdArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("c", I32),
                ("y", P), ("mem", P), ("stats", P), ("n", Neuron),
                ("g_out", P), ("g_state", P), ("pred_w", P), ("flow", P), ("g_flow", P),
                ("gflow_sb", I64), ("gflow_sc", I64),
                ("g_cur", P), ("g_mem", P), ("acc", P),
                ("zero0", P), ("zero1", P), ("zero_n", I32), ("mem_grad_in", I32)]


class LayerBwdArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("cin", I32), ("c", I32),
                ("y", P), ("stats", P), ("g_cur", P), ("acc_in", P), ("n", Neuron), ("ng", NeuronGrad),
                ("has_pred", I32), ("g_pred_w", P), ("g_pred_b", P), ("accumulate", I32),
                ("bnc_out", P), ("wt_bwd_ff", P), ("wt_bwd_rec", P),
                ("wt_fwd_ff", P), ("wt_fwd_rec", P), ("lif_in", I32),
                ("g_x", P), ("gxs_b", I64), ("gxs_c", I64), ("gxs_h", I64), ("gxs_w", I64),
                ("g_state_prev", P), ("zero_mem_half", I32),
                ("prev_y", P), ("prev_mem", P), ("prev_stats", P), ("prev", Neuron),
                ("prev_g_state", P), ("prev_g_cur", P), ("prev_g_mem", P), ("acc_out", P),
                ("zero0", P), ("zero1", P), ("zero_n", I32), ("wd_ff", P), ("wd_rec", P),
                ("wslab_ff", P), ("wslab_rec", P), ("s_prev", P), ("wslab_accumulate", I32),
                ("x", P), ("xs_b", I64), ("xs_c", I64), ("xs_h", I64), ("xs_w", I64)]


MAX_WGRAD_STEPS = 32


class WgradStep(ctypes.Structure):
    _fields_ = [("g_cur", P), ("y", P), ("x", P), ("xs_b", I64), ("xs_c", I64), ("xs_h", I64), ("xs_w", I64),
                ("s_prev", P), ("stats", P), ("bnc", P), ("x_bits", P), ("s_prev_bits", P)]


class WgradArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("cin", I32), ("c", I32), ("nsteps", I32),
                ("accumulate", I32), ("rec", I32), ("exact_inputs", I32), ("bn_weight", P), ("slab_ff", P),
                ("slab_rec", P),
                ("steps", WgradStep * MAX_WGRAD_STEPS)]


class ConvLifParams(ctypes.Structure):
    _fields_ = [("leak", P), ("thresh", P), ("act_width", F32), ("hard_reset", I32)]


class ConvLifFwdArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("cin", I32), ("c", I32),
                ("x", P), ("xs_b", I64), ("xs_c", I64), ("xs_h", I64), ("xs_w", I64),
                ("prev_state", P), ("wt_ff", P), ("wt_rec", P), ("p", ConvLifParams),
                ("residual", P), ("rs_b", I64), ("rs_c", I64), ("rs_h", I64), ("rs_w", I64),
                ("out", P), ("state", P), ("current", P)]


class ConvLifBwdArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("cin", I32), ("c", I32),
                ("g_out", P), ("gs_b", I64), ("gs_c", I64), ("gs_h", I64), ("gs_w", I64),
                ("g_state", P), ("state", P), ("prev_state", P), ("current", P),
                ("wt_bwd_ff", P), ("wt_bwd_rec", P), ("p", ConvLifParams),
                ("g_x", P), ("gxs_b", I64), ("gxs_c", I64), ("gxs_h", I64), ("gxs_w", I64),
                ("g_prev", P), ("g_current", P), ("acc", P)]


class EncodeArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("N", I32), ("H", I32), ("W", I32), ("ts", P), ("ys", P), ("xs", P), ("ps", P),
                ("ev_stride", I64), ("batch_stride", I64), ("num_bins", I32), ("round_ts", I32),
                ("accumulate", I32), ("cnt", P), ("voxel", P), ("image", P), ("mask", P), ("pol_mask", P)]


class AeeArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("flow", P), ("gtflow", P), ("event_mask", P),
                ("dt_ratio", P), ("flow_scaling", F32), ("acc", P), ("aee", P), ("percent", P),
                ("dt_gt", P), ("dt_input", P), ("dt_gt_n", I32), ("dt_input_n", I32)]


class FlowMetricsArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("flow", P), ("gtflow", P), ("event_mask", P),
                ("dt_ratio", P), ("flow_scaling", F32), ("mag_threshold", F32), ("rows", P), ("out", P)]


ADAM_MAX_TENSORS = 64  # SNNFLOW_ADAM_MAX_TENSORS
CLIP_ADAM_MAX_N = 1 << 20  # SNNFLOW_CLIP_ADAM_MAX_N


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", P), ("offset", I64), ("state_offset", I64), ("numel", I64)]


class ClipAdamArgs(ctypes.Structure):
    _fields_ = [("grad", P), ("exp_avg", P), ("exp_avg_sq", P), ("step", P), ("total_out", P), ("n", I64),
                ("lr", F64), ("beta1", F64), ("beta2", F64), ("eps", F64), ("weight_decay", F64),
                ("max_norm", F32), ("clip_eps", F32), ("ntensors", I32), ("t", AdamTensor * ADAM_MAX_TENSORS),
                ("scratch", P)]


# SNNFLOW_M_* output columns of snnflow_flow_metrics
METRICS = ("aee", "aee_pct", "nee", "nee_pct", "aae", "aae_pct", "naae", "ae_of_means", "aae_weighted",
           "aae_filtered")

ACC_SHARDS = 32  # SNNFLOW_ACC_SHARDS


def bwd_acc_len(c):
    """Sums per layer of the backward accumulator (SNNFLOW_BWD_ACC)."""
    return 5 * c + 2


def acc_storage(n):
    """Doubles occupied by a sharded accumulator of n sums (SNNFLOW_ACC_LEN)."""
    return ACC_SHARDS * ((n + 15) // 16 * 16)


class SlabDesc(ctypes.Structure):
    _fields_ = [("slab", P), ("out", P), ("elems", I32)]


class PrepDesc(ctypes.Structure):
    _fields_ = [("w", P), ("c", I32), ("cin", I32), ("wt_fwd", P), ("wt_bwd", P),
                ("threshold", P), ("thr_n", I32), ("frag_fwd", P), ("frag_bwd", P), ("zero", P), ("zero_n", I64)]


MAX_BATCH = 16


MAX_WINDOWS = 64


class IweLossArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("M", I32), ("T", I32), ("H", I32), ("W", I32), ("tf", I32),
                ("events", P * MAX_WINDOWS), ("pol", P * MAX_WINDOWS), ("flows", P * MAX_WINDOWS),
                ("masks", P * MAX_WINDOWS), ("off", ctypes.c_int32 * (MAX_WINDOWS + 1)),
                ("flow_scaling", F32), ("weight", F32),
                ("smoothing_mask", I32), ("overwrite_intermediate", I32), ("loss_scaling", I32),
                ("images", P), ("acc", P), ("persample", P), ("smooth", P), ("loss", P)]


UNET_MAX_SEGS = 4
UNET_MODE_S1, UNET_MODE_S2, UNET_MODE_T2 = 0, 1, 2
UNET_EPI_STORE, UNET_EPI_LIF = 0, 1
SURROGATES = {"arctanspike": 0, "superspike": 1, "mgspike": 2, "trianglespike": 3}


class UNetSeg(ctypes.Structure):
    _fields_ = [("x", P), ("H", I32), ("W", I32), ("cpitch", I32), ("mode", I32), ("kc0", I32), ("nparts", I32)]


class UNetConvArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("Ho", I32), ("Wo", I32), ("M", I32), ("ksize", I32), ("nseg", I32),
                ("seg", UNetSeg * UNET_MAX_SEGS), ("w", P), ("kct", I32), ("mpad", I32), ("xparts", I32),
                ("xpart", I64), ("pclass", I32), ("epi", I32),
                ("out", P), ("ld", I32), ("accumulate", I32),
                ("leak", P), ("thresh", P), ("hard_reset", I32), ("prev_state", P), ("residual", P),
                ("res_pitch", I32), ("state", P), ("current", P), ("act", P), ("act_pitch", I32),
                ("ksplit", I32), ("partial", P)]


class UNetWgradArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("Ho", I32), ("Wo", I32), ("M", I32), ("ksize", I32),
                ("g3", P), ("gpitch", I32), ("gpart", I64), ("seg", UNetSeg), ("k0", I32), ("ktot", I32),
                ("dwk", P), ("partial", P)]


class UNetLifBwdArgs(ctypes.Structure):
    _fields_ = [("P", I32), ("C", I32), ("leak", P), ("thresh", P), ("width", F32), ("hard_reset", I32),
                ("detach", I32), ("surrogate", I32), ("g_out", P), ("g_pitch", I32), ("g_state", P),
                ("state", P), ("prev_state", P), ("current", P), ("g_cur3", P), ("gc_pitch", I32),
                ("gc_part", I64), ("g_prev", P), ("g_res", P), ("gres_pitch", I32), ("acc", P), ("partial", P),
                ("res_assign", I32)]


MAX_LAYERS = 8
PL = P * MAX_LAYERS


class FireNetPlan(ctypes.Structure):
    _fields_ = [("L", I32), ("B", I32), ("H", I32), ("W", I32), ("c", I32), ("cin0", I32),
                ("rec", I32 * MAX_LAYERS), ("train", I32 * MAX_LAYERS), ("n", Neuron * MAX_LAYERS),
                ("wt_fwd_ff", PL), ("wt_fwd_rec", PL), ("wt_bwd_ff", PL), ("wt_bwd_rec", PL),
                ("wf_ff", PL), ("wf_rec", PL), ("wd_ff", PL), ("wd_rec", PL),
                ("fwd_acc", P), ("fwd_acc_stride", I64), ("bwd_acc", P), ("bwd_acc_stride", I64),
                ("pred_w", P), ("pred_b", P), ("slab_ff", PL), ("slab_rec", PL), ("nblk", I32)]


class FireNetFwdIo(ctypes.Structure):
    _fields_ = [("x", P), ("xs", I64 * 4), ("ys", P), ("stats", P), ("states", P), ("flow", P),
                ("mem_in", PL), ("s_prev", PL)]


class FireNetBwdIo(ctypes.Structure):
    _fields_ = [("ys", P), ("stats", P), ("flow", P), ("mem_in", PL), ("g_state", PL),
                ("g_flow", P), ("gflow_sb", I64), ("gflow_sc", I64), ("g_cur", P), ("bnc", P),
                ("g_prev", PL), ("ext", I32 * MAX_LAYERS), ("g_x", P), ("gxs", I64 * 4),
                ("ng", NeuronGrad * MAX_LAYERS), ("g_pred_w", P), ("g_pred_b", P), ("accumulate", I32)]


class FireNetSeqBwd(ctypes.Structure):
    _fields_ = [("T", I32), ("fresh", I32), ("fused", I32),
                ("ys", P * MAX_WINDOWS), ("stats", P * MAX_WINDOWS), ("flow", P * MAX_WINDOWS),
                ("states", P * MAX_WINDOWS), ("g_flow", P * MAX_WINDOWS),
                ("gflow_sb", I64 * MAX_WINDOWS), ("gflow_sc", I64 * MAX_WINDOWS),
                ("mem_in0", PL), ("s_prev0", PL), ("g_prev0", PL), ("ext0", I32 * MAX_LAYERS), ("g_state_last", PL),
                ("g_out", P), ("g_cur", P), ("bnc", P), ("bwd_acc", P), ("acc_stride", I64),
                ("ng", NeuronGrad * MAX_LAYERS), ("g_pred_w", P), ("g_pred_b", P),
                ("fuse_head", I32), ("x", P * MAX_WINDOWS), ("xs", (I64 * 4) * MAX_WINDOWS)]


class FireNetWgradStep(ctypes.Structure):
    _fields_ = [("g_cur", P), ("bnc", P), ("ys", P), ("stats", P), ("x", P), ("xs", I64 * 4), ("states", P),
                ("s_prev", PL)]


BN_PARTS = 256
ACT = {None: 0, "tanh": 1, "relu": 2, "sigmoid": 3}
PW_MAX_CIN, PW_MAX_COUT = 256, 4


class BnFwdArgs(ctypes.Structure):
    _fields_ = [("P", I64), ("C", I32), ("train", I32), ("x", P), ("y", P), ("weight", P), ("bias", P),
                ("running_mean", P), ("running_var", P), ("num_batches_tracked", P), ("momentum", F32), ("eps", F32),
                ("save_mean", P), ("save_invstd", P), ("scratch", P)]


class BnBwdArgs(ctypes.Structure):
    _fields_ = [("P", I64), ("C", I32), ("train", I32), ("x", P), ("g", P), ("weight", P), ("save_mean", P),
                ("save_invstd", P), ("g_x", P), ("g_weight", P), ("g_bias", P), ("scratch", P)]


class PointwiseArgs(ctypes.Structure):
    _fields_ = [("B", I32), ("H", I32), ("W", I32), ("cin", I32), ("cout", I32), ("act", I32), ("x", P),
                ("xs", I64 * 4), ("w", P), ("b", P), ("out", P), ("g_x", P), ("gxs", I64 * 4)]


EXPORTS = {
    "snnflow_abi_version": (I32, []),
    "snnflow_last_error": (ctypes.c_char_p, []),
    "snnflow_conv_blocks": (I32, [I32, I32, I32]),
    "snnflow_prep_weights": (I32, [P, I32, I32, P, P, P, P]),
    "snnflow_prep_weights_batch": (I32, [ctypes.POINTER(PrepDesc), I32, P]),
    "snnflow_conv_fwd": (I32, [ctypes.POINTER(ConvFwdArgs), P]),
    "snnflow_lif_fwd": (I32, [ctypes.POINTER(LifFwdArgs), P]),
    "snnflow_lif_bwd": (I32, [ctypes.POINTER(LifBwdArgs), P]),
    "snnflow_layer_bwd": (I32, [ctypes.POINTER(LayerBwdArgs), P]),
    "snnflow_wgrad": (I32, [ctypes.POINTER(WgradArgs), P]),
    "snnflow_convlif_fwd": (I32, [ctypes.POINTER(ConvLifFwdArgs), P]),
    "snnflow_encode_events": (I32, [ctypes.POINTER(EncodeArgs), P]),
    "snnflow_pol_iwe": (I32, [P, P, P, I64, I32, I32, I32, I32, I32, F32, F32, I32, P, P]),
    "snnflow_aee": (I32, [ctypes.POINTER(AeeArgs), P]),
    "snnflow_aee_acc_doubles": (I32, [I32, I32, I32]),
    "snnflow_flow_metrics": (I32, [ctypes.POINTER(FlowMetricsArgs), P]),
    "snnflow_flow_metrics_rows": (I32, [I32, I32, I32]),
    "snnflow_convlif_bwd": (I32, [ctypes.POINTER(ConvLifBwdArgs), P]),
    "snnflow_convlif_param_grads": (I32, [P, P, P, I32, I32, P, P, P]),
    "snnflow_slab_reduce": (I32, [ctypes.POINTER(SlabDesc), I32, I32, P]),
    "snnflow_iwe_loss_fwd": (I32, [ctypes.POINTER(IweLossArgs), P]),
    "snnflow_iwe_loss_bwd": (I32, [ctypes.POINTER(IweLossArgs), P, P, P]),
    "snnflow_device_errors": (I32, [I32]),
    "snnflow_iwe_scratch_floats": (I64, [I32, I32, I32, I32, I32, I32]),
    "snnflow_iwe_acc_doubles": (I32, [I32, I32, I32, I32]),
    "snnflow_iwe_corners": (I32, [P, P, I32, I32, F32, I32, I32, F32, I32, P, P, P]),
    "snnflow_iwe_interpolate": (I32, [P, P, P, I64, I32, I32, I32, I32, P, P]),
    "snnflow_iwe_corners_bwd": (I32, [P, P, I32, I32, F32, I32, I32, F32, P, P, P]),
    "snnflow_iwe_interpolate_bwd": (I32, [P, P, I64, I32, I32, I32, I32, P, P, P]),
    "snnflow_lif_export": (I32, [P, P, P, P, I32, I32, I32, P, P, P]),
    "snnflow_lif_theta_subtract": (I32, [P, P, P, I64, I32, P, P, P]),
    "snnflow_clip_grad_norm": (I32, [P, I64, F32, F32, P, P]),
    "snnflow_clip_grad_norm_large": (I32, [P, I64, F32, F32, P, P, P]),
    "snnflow_clip_adam": (I32, [P, P]),
    "snnflow_eval_slot": (I32, [P, I32, P]),
    "snnflow_count_nonzero": (I32, [P, P, I32, P, P]),
    "snnflow_fwd_slot": (I32, [ctypes.POINTER(ConvFwdArgs), I32, ctypes.POINTER(LifFwdArgs), P]),
    "snnflow_bwd_slot": (I32, [ctypes.POINTER(LayerBwdArgs), I32, ctypes.POINTER(LifBwdArgs), P]),
    "snnflow_slot_supported": (I32, [I32, I32]),
    "snnflow_set_pipe": (I32, [I32, I32]),
    "snnflow_get_pipe": (I32, [I32]),
    "snnflow_frag_halfs": (I32, [I32, I32]),
    "snnflow_unet_conv": (I32, [ctypes.POINTER(UNetConvArgs), P]),
    "snnflow_unet_conv_ksplit": (I32, [ctypes.POINTER(UNetConvArgs)]),
    "snnflow_unet_prep_weights": (I32, [P, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, P, P]),
    "snnflow_unet_wgrad": (I32, [ctypes.POINTER(UNetWgradArgs), P]),
    "snnflow_unet_wgrad_partial_floats": (I64, [ctypes.POINTER(UNetWgradArgs)]),
    "snnflow_unet_wgrad_finalize": (I32, [P, I32, P, I32, I32, I32, I32, I32, I32, P, P]),
    "snnflow_unet_lif_bwd": (I32, [ctypes.POINTER(UNetLifBwdArgs), P]),
    "snnflow_unet_lif_bwd_partial_doubles": (I32, [I32, I32, I32]),
    "snnflow_unet_cell_param_grads": (I32, [P, P, P, I32, I32, P, P, P]),
    "snnflow_unet_pack": (I32, [P, I32, I32, I32, I32, I64, I64, I64, I64, I32, P, I32, P]),
    "snnflow_unet_dec_in": (I32, [P, I32, I32, P, I32, I32, P, I32, I32, I32, P, I32, P]),
    "snnflow_unet_dec_in_bwd": (I32, [P, I32, I32, I32, I32, I32, I32, I32, P, I32, P, I32, P, I32, P]),
    "snnflow_unet_pred_fwd": (I32, [P, I32, I32, P, P, I32, I32, I32, I32, P, P, P]),
    "snnflow_unet_pred_bwd": (I32, [P, I32, I32, P, P, P, P, I32, I32, I32, I32, P, P, I32, P, I32, P, P]),
    "snnflow_unet_pred_bwd_partial_doubles": (I32, [I32, I32, I32, I32]),
    "snnflow_unet_pred_param_grads": (I32, [P, I32, I32, P, P, P]),
    "snnflow_firenet_fwd": (I32, [ctypes.POINTER(FireNetPlan), ctypes.POINTER(FireNetFwdIo), P]),
    "snnflow_firenet_bwd": (I32, [ctypes.POINTER(FireNetPlan), ctypes.POINTER(FireNetBwdIo), P]),
    "snnflow_firenet_bwd_seq": (I32, [ctypes.POINTER(FireNetPlan), ctypes.POINTER(FireNetSeqBwd), ctypes.POINTER(I32), P]),
    "snnflow_firenet_wgrad": (I32, [ctypes.POINTER(FireNetPlan), ctypes.POINTER(FireNetWgradStep), I32, P, P, P]),
    "snnflow_bn_fwd": (I32, [ctypes.POINTER(BnFwdArgs), P]),
    "snnflow_bn_bwd": (I32, [ctypes.POINTER(BnBwdArgs), P]),
    "snnflow_bn_scratch_doubles": (I32, [I32]),
    "snnflow_pointwise_fwd": (I32, [ctypes.POINTER(PointwiseArgs), P]),
    "snnflow_pointwise_bwd": (I32, [ctypes.POINTER(PointwiseArgs), P, I64, I64, P, P, P, P]),
}
MAX_SLOT_TASKS = 4
MAX_COUNT_TENSORS = 16


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"snnflow HIP library not found at {LIB_PATH}; build it with "
            "`make -C snn_event-based_optical_flow_amd/csrc` (or __graft_entry__.build()). "
            "There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.snnflow_abi_version() != ABI_VERSION:
        raise ImportError("snnflow ABI version mismatch; rebuild libsnnflow.so")
    return lib


lib = _load()


class SnnflowError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        raise SnnflowError(f"{what} failed ({rc}): {lib.snnflow_last_error().decode(errors='replace')}")


_DEVICE_FAULTS = {1: "event-warping forward: a bin segment outside its window's records (k_iwe_splat)",
                  2: "event-warping backward: a bin segment outside its window's records (k_iwe_bwd_band)"}


def check_device_errors(clear=True):
    """Raise SnnflowError if a kernel flagged (and skipped) a device-side argument fault since the last
    check -- e.g. a corrupted or stale loss scratch (snnflow_device_errors).  Synchronises the device."""
    rc = lib.snnflow_device_errors(1 if clear else 0)
    if rc < 0 or rc > 0xFFFF:
        check(rc, "device_errors")
    if rc:
        what = "; ".join(v for k, v in _DEVICE_FAULTS.items() if rc & k) or f"flags {rc:#x}"
        raise SnnflowError(f"device-side fault detected and skipped: {what}")


class KernelTimer:
    """Brackets C-ABI launches with HIP events on the launch stream (opt-in; used by bench.py to
    time the dominant kernel live).  records: list of (name, start, end, work, launches).

    The wavefront launches (GROUPED) come in runs of consecutive launches of one kernel (the 26
    forward or backward slots of a sequence): one event pair brackets the whole run and the run's
    time is divided by its launch count.  An event pair around every single launch would add the
    event commands' dispatch latency to each of these ~20-30 us kernels."""

    GROUPED = ("fwd_slot", "bwd_slot")

    def __init__(self):
        self.records = []
        self.open = None  # [name, start event, launches, work] of the run in progress

    def close(self):
        """End the open run of grouped launches (called before any other launch and by the
        engine right after a wavefront loop)."""
        if self.open is not None:
            name, a, n, work = self.open
            b = torch.cuda.Event(enable_timing=True)
            b.record()
            self.records.append((name, a, b, work, n))
            self.open = None

    def summary(self):
        self.close()
        torch.cuda.synchronize()
        out = {}
        for name, a, b, work, cnt in self.records:
            ms = a.elapsed_time(b)
            n, tot, w = out.get(name, (0, 0.0, 0.0))
            out[name] = (n + cnt, tot + ms, w + (work or 0.0))
        return {k: {"launches": n, "total_ms": tot, "avg_us": 1000.0 * tot / n, "work": w}
                for k, (n, tot, w) in out.items()}


TIMER = None


def timer_close():
    """Close the KernelTimer's open run of grouped launches (no-op without a timer)."""
    if TIMER is not None:
        TIMER.close()


def call(name, fn, *args, work=None):
    """Launch one C-ABI entry point; raise with the library's message on failure.  With a
    KernelTimer installed the launch is bracketed by HIP events on the current stream (runs of
    KernelTimer.GROUPED launches share one pair) and its algorithmic `work` (FLOPs, if given) is
    recorded with it."""
    if TIMER is None:
        check(fn(*args), name)
        return
    if name in TIMER.GROUPED:
        if TIMER.open is None or TIMER.open[0] != name:
            TIMER.close()
            a = torch.cuda.Event(enable_timing=True)
            a.record()
            TIMER.open = [name, a, 0, 0.0]
        check(fn(*args), name)
        TIMER.open[2] += 1
        TIMER.open[3] += work or 0.0
        return
    TIMER.close()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    check(fn(*args), name)
    b.record()
    TIMER.records.append((name, a, b, work, 1))


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


_HIP_SEEN = False  # a HIP device was visible once (torch.cuda.is_available() costs ~3 us a call)


def stream_ptr(device=None):
    """Raw HIP stream of the current stream on `device` (torch's getter without the Stream object)."""
    global _HIP_SEEN
    if not _HIP_SEEN:
        if not torch.cuda.is_available():
            raise SnnflowError("snnflow kernels need a HIP device (none visible); there is no CPU fallback")
        _HIP_SEEN = True
    if isinstance(device, str):
        device = torch.device(device)
    idx = device.index if isinstance(device, torch.device) else device
    if idx is None:
        idx = torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)


def require_device(t, name):
    if not t.is_cuda:
        raise SnnflowError(f"{name} must be a HIP device tensor (got {t.device}); there is no CPU fallback")
    if t.dtype != torch.float32:
        raise SnnflowError(f"{name} must be float32 (got {t.dtype})")
