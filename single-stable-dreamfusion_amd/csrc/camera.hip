// Camera rays of a full pinhole image as one launch (the per-step data path of
// the SDS loop: reference nerf/utils.py:42-106 get_rays with N = -1, called by
// nerf/provider.py:202-236 NeRFDataset.collate every train step).
//
// The reference builds the rays with ~10 torch ops per step (meshgrid,
// normalise, a batched 3x3 GEMM, expand).  Here the cam2world pose is passed
// by value (12 floats: the rotation rows and the centre), so the pose never
// touches device memory and the step's camera costs one kernel and no host
// synchronisation.  Arithmetic follows the torch expression order:
//   x = (i + 0.5 - cx) * (1/fx),  y = (j + 0.5 - cy) * (1/fy),  z = 1
//   d = v / sqrt(max(x*x + y*y + z*z, 1e-20))        (safe_normalize)
//   rays_d = R d  (row k: d0 R[k][0] + d1 R[k][1] + d2 R[k][2])
// The GEMM's summation order is the library's, so rays_d can differ from the
// torch version by an ulp (tests/test_gpu_camera.py bounds it).
#include "camera_common.h"

namespace dfhip {
namespace cam {

__global__ __launch_bounds__(256) void k_get_rays(Pose p, float fx, float fy, float cx,
                                                  float cy, uint32_t H, uint32_t W,
                                                  float *__restrict__ rays_o,
                                                  float *__restrict__ rays_d) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= H * W) return;
    float o[3], d[3];
    pixel_ray(p, fx, fy, cx, cy, W, n, o, d);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        rays_d[3 * (size_t)n + k] = d[k];
        rays_o[3 * (size_t)n + k] = o[k];
    }
}

}  // namespace cam
}  // namespace dfhip

using namespace dfhip;

extern "C" int dfhip_get_rays(const float *pose, float fx, float fy, float cx, float cy,
                              uint32_t H, uint32_t W, float *rays_o, float *rays_d,
                              dfhip_stream_t stream) {
    const char *name = "get_rays";
    if (!pose || !rays_o || !rays_d) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (!(fx != 0.0f) || !(fy != 0.0f)) {
        set_error("%s: focal lengths must be non-zero", name);
        return DFHIP_EINVAL;
    }
    const uint64_t n = (uint64_t)H * W;
    if (n == 0) return DFHIP_OK;
    if (n > 0xFFFFFFFFull) {
        set_error("%s: H*W too large", name);
        return DFHIP_EINVAL;
    }
    const cam::Pose p = cam::pose_from_3x4(pose);
    cam::k_get_rays<<<ceil_div((uint32_t)n, 256u), 256, 0, as_stream(stream)>>>(
        p, fx, fy, cx, cy, H, W, rays_o, rays_d);
    return check_launch(name);
}
