// pnraytracing_amd/csrc/pt_passes.h -- per-call passes shared by the
// integrators: the primary-hit pass (the primary ray has no jitter,
// ray_tracing.comp:980, so its closest hit is traced once per pnrt_render call
// and reused by every frame) and the frame-ordered progressive-mean blend
// (ray_tracing.comp:988-991).
#pragma once
#include "pt_path.h"

PN_DEV f3 camera_dir(const FrameParams& fp, int px, int py) {
    f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
    float sx = (float)px / (float)fp.width, sy = (float)py / (float)fp.height;
    return normalize(sub(add(add(mk3(fp.llc[0], fp.llc[1], fp.llc[2]), smul(sx, mk3(fp.hor[0], fp.hor[1], fp.hor[2]))),
                             smul(sy, mk3(fp.ver[0], fp.ver[1], fp.ver[2]))),
                         eye));
}

// ---- primary hits (once per call) ------------------------------------------------------------
// record: q0 = (P.xyz, bits(mat)), q1 = (N.xyz, u), q2 = (v, base.xyz); mat = -1 on a miss
// (base = emissive of the hit material, or the env colour of the primary direction)
__global__ void __launch_bounds__(256) pt_primary_kernel(DevScene s, FrameParams fp, float4* rec) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= fp.rows * fp.width) return;
    int lr = i / fp.width, px = i - lr * fp.width;
    int py = shard_row(lr, fp.band, fp.n_shards, fp.shard);
    f3 eye = mk3(fp.eye[0], fp.eye[1], fp.eye[2]);
    f3 dir = camera_dir(fp, px, py);
    RayP r = make_ray(eye, dir, fp.mode);
    float tmax = PT_FLOAT_MAX;
    int hitTri = -1;
    float4 q0, q1, q2;
    if (traverse<false>(s, r, tmax, hitTri)) {
        Hit h = make_hit(s, r, hitTri);
        f3 em = get_emissive(s, h.mat);
        q0 = make_float4(h.P.x, h.P.y, h.P.z, __int_as_float(h.mat));
        q1 = make_float4(h.N.x, h.N.y, h.N.z, h.u);
        q2 = make_float4(h.v, em.x, em.y, em.z);
        q0.w = __int_as_float((h.mat & 0x00ffffff) | ((h.tex + 1) << 24));   // mat < 2^24, tex in [-1,254]
    } else {
        f3 c = env_color(s, dir);
        q0 = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
        q1 = make_float4(0.f, 0.f, 0.f, 0.f);
        q2 = make_float4(0.f, c.x, c.y, c.z);
    }
    rec[3 * (size_t)i] = q0;
    rec[3 * (size_t)i + 1] = q1;
    rec[3 * (size_t)i + 2] = q2;
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
