// Event warp and bilinear corners shared by the loss and evaluation kernels
// (utils/iwe.py:20-71 get_interpolation + purge_unfeasible; bit-exactness contract in
// iwe_loss.hip's header comment).
#pragma once

#include "snnflow_dev.h"

namespace snnflow {

struct Corner {
    int idx;      // flat pixel index (0 when out of bounds, like purge_unfeasible)
    bool inb;
    float ay, ax; // per-axis bilinear factors max(0, 1-|w-c|)
    float dy, dx; // w - c per axis
    float wt;     // ay*ax*inb
};

// get_interpolation for one event and one reference time (4 corners, corner-major order).
__device__ inline void warp4(float ts, float y, float x, float fy, float fx, float tref, float s, int H, int W,
                             Corner (&c)[4], float& wy, float& wx) {
    const float dt = tref - ts;
    wy = y + (dt * fy) * s;
    wx = x + (dt * fx) * s;
    const float y0 = floorf(wy), y1 = floorf(wy + 1.0f);
    const float x0 = floorf(wx), x1 = floorf(wx + 1.0f);
    const float cy[4] = {y0, y0, y1, y1}, cx[4] = {x0, x1, x0, x1};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool inb = (cy[k] >= 0.0f) && (cy[k] < (float)H) && (cx[k] >= 0.0f) && (cx[k] < (float)W);
        const float m = inb ? 1.0f : 0.0f;
        c[k].inb = inb;
        c[k].dy = wy - cy[k];
        c[k].dx = wx - cx[k];
        c[k].ay = fmaxf(0.0f, 1.0f - fabsf(c[k].dy));
        c[k].ax = fmaxf(0.0f, 1.0f - fabsf(c[k].dx));
        c[k].wt = (c[k].ay * c[k].ax) * m;
        c[k].idx = (int)((cy[k] * m) * (float)W + cx[k] * m);
    }
}

}  // namespace snnflow
