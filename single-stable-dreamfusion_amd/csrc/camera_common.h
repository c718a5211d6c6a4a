// Pinhole camera rays shared by the get_rays launch (camera.hip) and the
// train-step prologue (step.hip).  Reference nerf/utils.py:42-106 (get_rays,
// N = -1); arithmetic in the torch expression order (see camera.hip).
#pragma once

#include "common.h"

namespace dfhip {
namespace cam {

struct Pose {
    float r[9];  // rotation, row-major (cam2world[:3, :3])
    float t[3];  // centre (cam2world[:3, 3])
};

// Ray of pixel n = h * W + w: origin o, direction d (safe-normalised camera
// direction rotated into the world).
__device__ __forceinline__ void pixel_ray(const Pose &p, float fx, float fy, float cx, float cy,
                                          uint32_t W, uint32_t n, float o[3], float d[3]) {
    const uint32_t h = n / W, w = n - h * W;
    // torch divides a tensor by a scalar as a multiply by its f32 reciprocal
    const float x = ((float)w + 0.5f - cx) * (1.0f / fx);
    const float y = ((float)h + 0.5f - cy) * (1.0f / fy);
    const float s = (x * x + y * y) + 1.0f;
    const float inv = sqrtf(fmaxf(s, 1e-20f));
    const float d0 = x / inv, d1 = y / inv, d2 = 1.0f / inv;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        d[k] = fmaf(d2, p.r[3 * k + 2], fmaf(d1, p.r[3 * k + 1], d0 * p.r[3 * k]));
        o[k] = p.t[k];
    }
}

inline Pose pose_from_3x4(const float *pose) {
    Pose p;
    for (int k = 0; k < 3; ++k) {
        for (int c = 0; c < 3; ++c) p.r[3 * k + c] = pose[4 * k + c];
        p.t[k] = pose[4 * k + 3];
    }
    return p;
}

}  // namespace cam
}  // namespace dfhip
