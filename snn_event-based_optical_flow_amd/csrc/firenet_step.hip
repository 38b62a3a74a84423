// Host-side driver of one LIFFireNet time step (forward / backward) and of a BPTT window's deferred
// weight gradients: builds the kernel arguments of snnflow_conv_fwd / snnflow_lif_fwd /
// snnflow_lif_bwd / snnflow_layer_bwd / snnflow_wgrad / snnflow_slab_reduce from a per-model plan
// and per-step pointers, so that the eager drop-in loop (one model() call per window,
// train_flow.py:231-279) pays one library call per time step and direction instead of building
// about twenty argument structs in Python.  The accumulator hand-over (which kernel zeroes which
// batch-sum accumulator) is the chain order of snnflow/engine.py FireNetStep.
#include <cstring>

#include "snnflow_dev.h"

int snnflow_set_error(int code, const char* msg);
#define SNN_FAIL(code, msg) return snnflow_set_error((code), (msg))

namespace {

inline int check_plan(const snnflow_firenet_plan* p) {
    if (!p || p->L < 1 || p->L > SNNFLOW_MAX_LAYERS || p->B <= 0 || p->H <= 0 || p->W <= 0 || p->c <= 0 ||
        p->cin0 <= 0 || !p->fwd_acc || !p->bwd_acc)
        return -1;
    return 0;
}

inline const float* spike_half(const float* state, const snnflow_firenet_plan* p) {
    return state + (int64_t)p->B * p->H * p->W * p->c;
}

}  // namespace

extern "C" {

int snnflow_firenet_fwd(const snnflow_firenet_plan* p, const snnflow_firenet_fwd_io* io, void* stream) {
    if (check_plan(p) || !io || !io->x || !io->ys || !io->stats || !io->states || !io->flow)
        SNN_FAIL(SNNFLOW_E_ARG, "firenet_fwd: bad arguments");
    const int L = p->L, C = p->c;
    const int64_t npix = (int64_t)p->B * p->H * p->W;
    const int64_t ny = npix * C, nst = 2 * npix * C;
    const int zn = (int)p->fwd_acc_stride;
    for (int l = 0; l < L; ++l) {
        snnflow_conv_fwd_args a;
        memset(&a, 0, sizeof(a));
        a.B = p->B; a.H = p->H; a.W = p->W; a.c = C;
        if (l == 0) {
            a.cin = p->cin0; a.lif_in = 0;
            a.x = io->x;
            a.xs_b = io->xs[0]; a.xs_c = io->xs[1]; a.xs_h = io->xs[2]; a.xs_w = io->xs[3];
            a.zero0 = p->fwd_acc + (int64_t)(L - 1) * p->fwd_acc_stride;
            a.zero_n = zn;
        } else {
            a.cin = C; a.lif_in = 1;
            a.prev_y = io->ys + (l - 1) * ny;
            a.prev_mem = io->mem_in[l - 1];
            a.prev_acc = p->fwd_acc + (int64_t)(l - 1) * p->fwd_acc_stride;
            a.prev_stats = io->stats + (int64_t)(l - 1) * 2 * C;
            a.prev = p->n[l - 1];
            a.prev_state = io->states + (l - 1) * nst;
            if (l >= 2) {
                a.zero0 = p->fwd_acc + (int64_t)(l - 2) * p->fwd_acc_stride;
                a.zero_n = zn;
            }
        }
        a.wt_ff = p->wt_fwd_ff[l]; a.wt_rec = p->wt_fwd_rec[l];
        a.wt_ff_t = p->wt_bwd_ff[l]; a.wt_rec_t = p->wt_bwd_rec[l];
        a.s_prev = io->s_prev[l];
        a.y = io->ys + l * ny;
        a.acc = p->train[l] ? p->fwd_acc + (int64_t)l * p->fwd_acc_stride : nullptr;
        a.wf_ff = p->wf_ff[l]; a.wf_rec = p->wf_rec[l];
        int rc = snnflow_conv_fwd(&a, stream);
        if (rc) return rc;
    }
    snnflow_lif_fwd_args f;
    memset(&f, 0, sizeof(f));
    f.B = p->B; f.H = p->H; f.W = p->W; f.c = C;
    f.y = io->ys + (L - 1) * ny;
    f.mem = io->mem_in[L - 1];
    f.acc = p->fwd_acc + (int64_t)(L - 1) * p->fwd_acc_stride;
    f.stats = io->stats + (int64_t)(L - 1) * 2 * C;
    f.n = p->n[L - 1];
    f.state = io->states + (L - 1) * nst;
    f.pred_w = p->pred_w; f.pred_b = p->pred_b; f.flow = io->flow;
    if (L >= 2) {
        f.zero0 = p->fwd_acc + (int64_t)(L - 2) * p->fwd_acc_stride;
        f.zero_n = zn;
    }
    return snnflow_lif_fwd(&f, stream);
}

int snnflow_firenet_bwd(const snnflow_firenet_plan* p, const snnflow_firenet_bwd_io* io, void* stream) {
    if (check_plan(p) || !io || !io->ys || !io->stats || !io->flow || !io->g_cur || !io->bnc)
        SNN_FAIL(SNNFLOW_E_ARG, "firenet_bwd: bad arguments");
    const int L = p->L, C = p->c, top = L - 1;
    const int64_t npix = (int64_t)p->B * p->H * p->W;
    const int64_t ny = npix * C;
    const int zn = (int)p->bwd_acc_stride;
    // gradients flowing into the membrane input: only for states this model did not produce
    float* g_mem[SNNFLOW_MAX_LAYERS];
    for (int l = 0; l < L; ++l) g_mem[l] = (io->g_prev[l] && io->ext[l]) ? io->g_prev[l] : nullptr;

    snnflow_lif_bwd_args b;
    memset(&b, 0, sizeof(b));
    b.B = p->B; b.H = p->H; b.W = p->W; b.c = C;
    b.y = io->ys + top * ny; b.mem = io->mem_in[top]; b.stats = io->stats + (int64_t)top * 2 * C; b.n = p->n[top];
    b.g_state = io->g_state[top];
    b.pred_w = p->pred_w; b.flow = io->flow;
    if (io->g_flow) {
        b.g_flow = io->g_flow; b.gflow_sb = io->gflow_sb; b.gflow_sc = io->gflow_sc;
    }
    b.g_cur = io->g_cur + top * ny; b.g_mem = g_mem[top];
    b.acc = p->bwd_acc + (int64_t)top * p->bwd_acc_stride;
    b.zero0 = p->bwd_acc;
    b.zero_n = zn;
    int rc = snnflow_lif_bwd(&b, stream);
    if (rc) return rc;

    for (int l = L - 1; l >= 0; --l) {
        snnflow_layer_bwd_args a;
        memset(&a, 0, sizeof(a));
        a.B = p->B; a.H = p->H; a.W = p->W; a.c = C;
        a.y = io->ys + l * ny; a.stats = io->stats + (int64_t)l * 2 * C; a.g_cur = io->g_cur + l * ny;
        a.acc_in = p->bwd_acc + (int64_t)l * p->bwd_acc_stride;
        a.n = p->n[l];
        a.ng = io->ng[l];
        a.accumulate = io->accumulate;
        a.bnc_out = io->bnc + (int64_t)l * 2 * C;
        if (l == L - 1) {
            a.has_pred = 1; a.g_pred_w = io->g_pred_w; a.g_pred_b = io->g_pred_b;
        }
        if (p->rec[l]) {
            a.wt_bwd_rec = p->wt_bwd_rec[l]; a.wt_fwd_rec = p->wt_fwd_rec[l];
            if (io->g_prev[l]) {
                a.g_state_prev = io->g_prev[l];
                a.zero_mem_half = io->ext[l] ? 0 : 1;
            }
        }
        a.wd_ff = p->wd_ff[l]; a.wd_rec = p->wd_rec[l];
        if (l > 0) {
            a.cin = C; a.lif_in = 1;
            a.wt_bwd_ff = p->wt_bwd_ff[l]; a.wt_fwd_ff = p->wt_fwd_ff[l];
            a.prev_y = io->ys + (l - 1) * ny; a.prev_mem = io->mem_in[l - 1];
            a.prev_stats = io->stats + (int64_t)(l - 1) * 2 * C; a.prev = p->n[l - 1];
            a.prev_g_state = io->g_state[l - 1];
            a.prev_g_cur = io->g_cur + (l - 1) * ny; a.prev_g_mem = g_mem[l - 1];
            a.acc_out = p->bwd_acc + (int64_t)(l - 1) * p->bwd_acc_stride;
        } else {
            a.cin = p->cin0; a.lif_in = 0;
            if (io->g_x) {
                a.wt_bwd_ff = p->wt_bwd_ff[0]; a.wt_fwd_ff = p->wt_fwd_ff[0];
                a.g_x = io->g_x;
                a.gxs_b = io->gxs[0]; a.gxs_c = io->gxs[1]; a.gxs_h = io->gxs[2]; a.gxs_w = io->gxs[3];
            }
        }
        if (l + 1 <= L - 1) {
            a.zero0 = p->bwd_acc + (int64_t)(l + 1) * p->bwd_acc_stride;
            a.zero_n = zn;
        }
        rc = snnflow_layer_bwd(&a, stream);
        if (rc) return rc;
    }
    return 0;
}

int snnflow_firenet_bwd_seq(const snnflow_firenet_plan* p, const snnflow_firenet_seq_bwd* q, int* slab_live,
                            void* stream) {
    if (check_plan(p) || !q || q->T < 1 || q->T > SNNFLOW_MAX_WINDOWS || !q->bwd_acc || !q->g_cur || !q->bnc ||
        q->acc_stride < SNNFLOW_ACC_LEN(SNNFLOW_BWD_ACC(p->c)) || !slab_live)
        SNN_FAIL(SNNFLOW_E_ARG, "firenet_bwd_seq: bad arguments");
    const int L = p->L, C = p->c, top = L - 1, K = L + 1, T = q->T;
    if (q->fused && C != 8) SNN_FAIL(SNNFLOW_E_ARG, "firenet_bwd_seq: fused weight gradients need c = 8");
    const int64_t npix = (int64_t)p->B * p->H * p->W;
    const int64_t ny = npix * C, nst = 2 * ny;
    int rslot[SNNFLOW_MAX_LAYERS], nrec = 0;  // recurrent layer -> its g_out slot within a step
    for (int l = 0; l < L; ++l) rslot[l] = p->rec[l] ? nrec++ : -1;
    if (T > 1 && nrec && !q->g_out) SNN_FAIL(SNNFLOW_E_ARG, "firenet_bwd_seq: g_out missing");
    for (int t = 0; t < T; ++t)
        if (!q->ys[t] || !q->stats[t] || !q->flow[t] || !q->states[t] || (q->fuse_head && !q->x[t]))
            SNN_FAIL(SNNFLOW_E_ARG, "firenet_bwd_seq: incomplete step");
    if (q->fuse_head && (p->rec[0] || !(p->cin0 == 2 || p->cin0 == 4) || !p->slab_ff[0]))
        SNN_FAIL(SNNFLOW_E_ARG, "firenet_bwd_seq: fuse_head needs a feed-forward 2- or 4-channel head and its slab");
    // every launch's layer-task count, checked before the first launch (the call refuses cleanly or runs
    // to completion: no half-written gradients or slab rows)
    for (int d = 0; d < K + 2 * (T - 1); ++d) {
        int n = 0;
        for (int j = 1; j < K; ++j)
            if ((d - j) >= 0 && (d - j) % 2 == 0 && (d - j) / 2 < T) ++n;
        if (n > SNNFLOW_MAX_SLOT_TASKS) SNN_FAIL(SNNFLOW_E_ARG, "firenet_bwd_seq: too many layers for a launch");
    }
    // gradient of step t's incoming state of layer l (t >= 1: inside the chain, recurrent layers only)
    auto g_in = [&](int t, int l) -> float* {
        if (t == 0) return q->g_prev0[l];
        return rslot[l] >= 0 ? q->g_out + ((int64_t)(t - 1) * nrec + rslot[l]) * nst : nullptr;
    };
    // gradient flowing into step t's output state of layer l
    auto g_st = [&](int t, int l) -> const float* { return t == T - 1 ? q->g_state_last[l] : g_in(t + 1, l); };
    auto mem_in = [&](int t, int l) -> const float* { return t == 0 ? q->mem_in0[l] : q->states[t - 1] + l * nst; };
    auto s_prev = [&](int t, int l) -> const float* {
        return t == 0 ? q->s_prev0[l] : (p->rec[l] ? q->states[t - 1] + l * nst + ny : nullptr);
    };
    auto acc_of = [&](int t, int l) { return q->bwd_acc + ((int64_t)t * L + l) * q->acc_stride; };
    for (int d = 0; d < K + 2 * (T - 1); ++d) {
        snnflow_layer_bwd_args la[SNNFLOW_MAX_SLOT_TASKS];
        snnflow_lif_bwd_args tb;
        int nl = 0;
        bool has_top = false;
        for (int j = 0; j < K; ++j) {
            if ((d - j) % 2 || (d - j) < 0 || (d - j) / 2 >= T) continue;
            const int t = T - 1 - (d - j) / 2;
            const float* ys = q->ys[t];
            const float* stats = q->stats[t];
            float* gcur = q->g_cur + (int64_t)t * L * ny;
            auto g_mem = [&](int l) -> float* { return (t == 0 && q->ext0[l] && q->g_prev0[l]) ? q->g_prev0[l] : nullptr; };
            if (j == 0) {  // pred backward + LIF backward of layer L-1
                snnflow_lif_bwd_args& b = tb;
                memset(&b, 0, sizeof(b));
                b.B = p->B; b.H = p->H; b.W = p->W; b.c = C;
                b.y = ys + top * ny; b.mem = mem_in(t, top); b.stats = stats + (int64_t)top * 2 * C; b.n = p->n[top];
                b.g_state = g_st(t, top);
                b.pred_w = p->pred_w; b.flow = q->flow[t];
                if (q->g_flow[t]) {
                    b.g_flow = q->g_flow[t]; b.gflow_sb = q->gflow_sb[t]; b.gflow_sc = q->gflow_sc[t];
                }
                b.g_cur = gcur + top * ny; b.g_mem = g_mem(top);
                b.acc = acc_of(t, top);
                has_top = true;
                continue;
            }
            const int l = L - j;
            if (nl == SNNFLOW_MAX_SLOT_TASKS) SNN_FAIL(SNNFLOW_E_ARG, "firenet_bwd_seq: too many layers for a launch");
            snnflow_layer_bwd_args& a = la[nl++];
            memset(&a, 0, sizeof(a));
            a.B = p->B; a.H = p->H; a.W = p->W; a.c = C;
            a.y = ys + l * ny; a.stats = stats + (int64_t)l * 2 * C; a.g_cur = gcur + l * ny;
            a.acc_in = acc_of(t, l);
            a.n = p->n[l];
            a.ng = q->ng[l];
            a.accumulate = (q->fresh && t == T - 1) ? 0 : 1;
            a.bnc_out = q->bnc + ((int64_t)t * L + l) * 2 * C;
            if (l == L - 1) {
                a.has_pred = 1; a.g_pred_w = q->g_pred_w; a.g_pred_b = q->g_pred_b;
            }
            if (p->rec[l]) {
                a.wt_bwd_rec = p->wt_bwd_rec[l]; a.wt_fwd_rec = p->wt_fwd_rec[l];
                if (float* gp = g_in(t, l)) {
                    a.g_state_prev = gp;
                    // steps t >= 1: the gradient stays inside the chain and its membrane half is never
                    // read (the cells detach the reset); step 0's leaves the chain zero-filled
                    a.zero_mem_half = (t == 0 && !q->ext0[l]) ? 1 : 0;
                }
            }
            a.wd_ff = p->wd_ff[l]; a.wd_rec = p->wd_rec[l];
            if (l > 0) {
                a.cin = C; a.lif_in = 1;
                a.wt_bwd_ff = p->wt_bwd_ff[l]; a.wt_fwd_ff = p->wt_fwd_ff[l];
                a.prev_y = ys + (l - 1) * ny; a.prev_mem = mem_in(t, l - 1);
                a.prev_stats = stats + (int64_t)(l - 1) * 2 * C; a.prev = p->n[l - 1];
                a.prev_g_state = g_st(t, l - 1);
                a.prev_g_cur = gcur + (l - 1) * ny; a.prev_g_mem = g_mem(l - 1);
                a.acc_out = acc_of(t, l - 1);
                if (q->fused) {
                    a.wslab_ff = p->slab_ff[l];
                    if (p->rec[l]) {
                        a.wslab_rec = p->slab_rec[l];
                        a.s_prev = s_prev(t, l);
                    }
                    a.wslab_accumulate = slab_live[l] ? 1 : 0;
                    slab_live[l] = 1;
                }
            } else {
                a.cin = p->cin0; a.lif_in = 0;
                if (q->fuse_head) {  // ABI 40: the head's weight gradient of step t in this task
                    a.x = q->x[t];
                    a.xs_b = q->xs[t][0]; a.xs_c = q->xs[t][1]; a.xs_h = q->xs[t][2]; a.xs_w = q->xs[t][3];
                    a.wslab_ff = p->slab_ff[0];
                    a.wslab_accumulate = slab_live[0] ? 1 : 0;
                    slab_live[0] = 1;
                }
            }
        }
        const int rc = snnflow_bwd_slot(la, nl, has_top ? &tb : nullptr, stream);
        if (rc) return rc;
    }
    return 0;
}

int snnflow_firenet_wgrad(const snnflow_firenet_plan* p, const snnflow_firenet_wgrad_step* steps, int nsteps,
                          float* const* g_ff, float* const* g_rec, void* stream) {
    if (check_plan(p) || !steps || nsteps < 1 || !g_ff || p->nblk <= 0)
        SNN_FAIL(SNNFLOW_E_ARG, "firenet_wgrad: bad arguments");
    const int L = p->L, C = p->c;
    const int64_t npix = (int64_t)p->B * p->H * p->W;
    const int64_t ny = npix * C;
    snnflow_wgrad_args a;  // ~3 KB (32 steps)
    for (int l = 0; l < L; ++l) {
        if (!p->slab_ff[l] || (p->rec[l] && !p->slab_rec[l])) SNN_FAIL(SNNFLOW_E_ARG, "firenet_wgrad: slabs");
        for (int i0 = 0; i0 < nsteps; i0 += SNNFLOW_MAX_WGRAD_STEPS) {
            const int n = nsteps - i0 < SNNFLOW_MAX_WGRAD_STEPS ? nsteps - i0 : SNNFLOW_MAX_WGRAD_STEPS;
            memset(&a, 0, sizeof(a));
            a.B = p->B; a.H = p->H; a.W = p->W; a.c = C;
            a.cin = l == 0 ? p->cin0 : C;
            a.nsteps = n; a.accumulate = i0 ? 1 : 0; a.rec = p->rec[l];
            a.exact_inputs = l > 0 ? 1 : 0;   // layers >= 1 read this model's spikes (exact in bf16)
            a.bn_weight = p->n[l].bn_weight;
            a.slab_ff = p->slab_ff[l]; a.slab_rec = p->slab_rec[l];
            for (int k = 0; k < n; ++k) {
                const snnflow_firenet_wgrad_step& s = steps[i0 + k];
                snnflow_wgrad_step& st = a.steps[k];
                st.g_cur = s.g_cur + l * ny; st.y = s.ys + l * ny;
                st.stats = s.stats + (int64_t)l * 2 * C; st.bnc = s.bnc + (int64_t)l * 2 * C;
                if (l == 0) {
                    st.x = s.x;
                    st.xs_b = s.xs[0]; st.xs_c = s.xs[1]; st.xs_h = s.xs[2]; st.xs_w = s.xs[3];
                } else {  // spike half of the previous layer's state, NHWC
                    st.x = spike_half(s.states + (l - 1) * 2 * ny, p);
                    st.xs_b = (int64_t)p->H * p->W * C; st.xs_c = 1; st.xs_h = (int64_t)p->W * C; st.xs_w = C;
                }
                st.s_prev = p->rec[l] ? s.s_prev[l] : nullptr;
            }
            int rc = snnflow_wgrad(&a, stream);
            if (rc) return rc;
        }
    }
    snnflow_slab_desc d[SNNFLOW_MAX_SLABS];
    int nd = 0;
    for (int l = 0; l < L; ++l) {
        const int cin = l == 0 ? p->cin0 : C;
        d[nd].slab = p->slab_ff[l]; d[nd].out = g_ff[l]; d[nd].elems = C * cin * 9; ++nd;
        if (p->rec[l]) {
            d[nd].slab = p->slab_rec[l]; d[nd].out = g_rec[l]; d[nd].elems = C * C * 9; ++nd;
        }
        if (nd > SNNFLOW_MAX_SLABS - 2 || l == L - 1) {
            int rc = snnflow_slab_reduce(d, nd, p->nblk, stream);
            if (rc) return rc;
            nd = 0;
        }
    }
    return 0;
}

}  // extern "C"
