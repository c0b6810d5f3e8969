"""Native operator bindings (HIP kernels for gfx950, C++ GBDT engine)."""
