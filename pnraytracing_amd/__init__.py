"""pnraytracing_amd -- MI355X-native replacement of PnRayTracing's radiance
integrator (shaders/ray_tracing.comp) behind a C ABI (include/pnrt.h).

    host      -- scene arrays bit-identical to main.cpp's uploads (libpnrt_host.so)
    scenes    -- benchmark/parity configurations C1-C5
    tracer    -- PathTracer over the HIP library (libpnrt.so)
    dist      -- one process per GPU, row-band sharding + RCCL gather
"""
__version__ = "0.1.0"
