// kb_build_tu.hip -- the build kernels (k_build / k_buildp) of ONE camera-model set, in a translation unit of their
// own: the library compiles the nine model sets in parallel instead of instantiating ~100 large kernels in kb_capi.hip.
// Compiled with -DKB_TU_ID=<0..8>; kb_capi.hip's pick_build dispatches to kb_build_fn_<id>.  kb_kernels.hip is
// included inside an unnamed namespace, so the non-template kernels it also defines stay internal to this TU (the
// copies nothing here references are not emitted twice into one symbol).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kalibr_hip.h"

namespace {
#include "kb_kernels.hip"

#ifndef KB_TU_ID
#error "KB_TU_ID (0..8) selects the camera-model set"
#endif
constexpr unsigned kTuMm[9] = {1u << KB_PINHOLE_RADTAN, 1u << KB_OMNI_RADTAN, 1u << KB_EUCM, 1u << KB_OMNI,
                               1u << KB_DS, 1u << KB_PINHOLE_EQUI, 1u << KB_PINHOLE_FOV,
                               (1u << KB_OMNI_RADTAN) | (1u << KB_EUCM), kb::kMmAll};
constexpr unsigned MM = kTuMm[KB_TU_ID];

// mb: Schur tiles per wave of k_build (1 | 4 | 7), or per frame wave of k_buildp (5: 2 frame waves | 7: 4) when pipe
template <bool GN>
const void* build_fn(int mb, bool pipe, bool wide) {
  using namespace kb;
  constexpr int MWN = kBuildpMaxCams + 4;
  if constexpr (__builtin_popcount(MM) >= 2) {  // multi-model view roles: the spill-free 8-wave variant
    if (pipe && wide) return mb == 5 ? (const void*)k_buildp<5, GN, MM, 8> : (const void*)k_buildp<7, GN, MM, 8>;
  }
  if (pipe) return mb == 5 ? (const void*)k_buildp<5, GN, MM, MWN> : (const void*)k_buildp<7, GN, MM, MWN>;
  return mb == 1 ? (const void*)k_build<1, GN, MM> : mb == 4 ? (const void*)k_build<4, GN, MM>
                                                             : (const void*)k_build<7, GN, MM>;
}
}  // namespace

#define KB_CAT2(a, b) a##b
#define KB_CAT(a, b) KB_CAT2(a, b)
const void* KB_CAT(kb_build_fn_, KB_TU_ID)(bool gn, int mb, bool pipe, bool wide) {
  return gn ? build_fn<true>(mb, pipe, wide) : build_fn<false>(mb, pipe, wide);
}
