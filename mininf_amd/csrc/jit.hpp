// Interface between the launch planner (sites.hip) and the site-program specialiser (jit.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "mininf_amd.h"

struct PlanInfo {
  bool row;        // lanes along elements (true) or along particles (false)
  int elems;       // ROW: elements per lane per row; COL: unroll of the element loop
  int kw;          // COL: lanes per element group (power of two <= 64)
  bool combined;   // reduce one weighted log-joint value per particle instead of one per site
  bool block_rows; // fused-draw row loop: one partial row per block (gridDim.x rows), not per wave
  bool packed;     // fused-draw row loop: element pairs on packed fp32 math where the families allow
  unsigned grid_x;
  unsigned grid_y;
};

// Launch the specialised kernel for `g` (compiling it on first use). Returns 0 on success, 1 if
// specialisation is unavailable (disabled or failed to compile: the caller uses the generic
// kernel), or a negative hipError_t.
int mi_jit_launch(const mi_group& g, const PlanInfo& plan, float* part, int64_t nseg, int64_t arg,
                  uint32_t* flags, hipStream_t stream);

// Generated source for inspection and tests.
std::string mi_jit_source(const mi_group& g, const PlanInfo& plan);

size_t mi_jit_cache_size();

// Whether specialised kernels are compiled at all (MININF_AMD_JIT=0 disables them).
bool mi_jit_enabled();

// Compile (hiprtc only, no device needed) the specialised kernel for `g`; returns success and the
// compiler log.
bool mi_jit_compile_check(const mi_group& g, const PlanInfo& plan, std::string* log);
