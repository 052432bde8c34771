// pnraytracing_amd/csrc/pt_passes.h -- per-call pieces shared by the
// integrators: the camera ray (CameraGetRay, ray_tracing.comp:205-211) and the
// frame-ordered progressive-mean blend (ray_tracing.comp:988-991).  The primary
// pass itself is pt_wf.h pt_primary_wf.
#pragma once
#include "pt_path.h"

PN_DEV f3 camera_dir(const FrameParams& fp, int px, int py) {
    f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
    float sx = (float)px / (float)fp.width, sy = (float)py / (float)fp.height;
    return normalize(sub(add(add(mk3(fp.llc[0], fp.llc[1], fp.llc[2]), smul(sx, mk3(fp.hor[0], fp.hor[1], fp.hor[2]))),
                             smul(sy, mk3(fp.ver[0], fp.ver[1], fp.ver[2]))),
                         eye));
}

// Frame-ordered progressive mean (ray_tracing.comp:988-991) of one chunk.
__global__ void pt_blend_kernel(FrameParams fp, const float4* colors, float4* accum, int chunk_frames,
                                uint32_t first_frame) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= fp.rows * fp.width) return;
    int lr = i / fp.width, px = i - lr * fp.width;
    int py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
    size_t pix = (size_t)py * fp.width + px;
    float4 acc = accum[pix];
    for (int k = 0; k < chunk_frames; ++k) {
        float4 c = colors[((size_t)k * fp.rows + lr) * fp.width + px];
        float a = 1.0f / (float)(first_frame + (uint32_t)k + 1u);
        acc.x = mixf(acc.x, c.x, a);
        acc.y = mixf(acc.y, c.y, a);
        acc.z = mixf(acc.z, c.z, a);
        acc.w = 1.0f;
    }
    accum[pix] = acc;
}
