// ABI bookkeeping entry points of libdexiraft_corr.so (include/dexiraft_corr.h).
#include "dxr_common.h"

namespace dxr {
namespace {
thread_local int g_last_hip_error = 0;
}
void set_last_hip_error(hipError_t e) { g_last_hip_error = (int)e; }
}  // namespace dxr

extern "C" int dxr_abi_version(void) { return DXR_ABI_VERSION; }

extern "C" const char* dxr_status_string(int status) {
  switch (status) {
    case DXR_OK: return "ok";
    case DXR_EINVAL: return "invalid argument";
    case DXR_EUNSUPPORTED: return "unsupported by this build";
    case DXR_EHIP: return "HIP launch error";
    default: return "unknown status";
  }
}

extern "C" int dxr_last_hip_error(void) { return dxr::g_last_hip_error; }

extern "C" int64_t dxr_pyramid_numel(int64_t B, int64_t H, int64_t W, int num_levels) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return -1;
  return L.numel;
}

extern "C" int64_t dxr_pyramid_level_offset(int64_t B, int64_t H, int64_t W, int level) {
  dxr::Levels L;
  if (level < 0 || !dxr::make_levels(B, H, W, level + 1, &L)) return -1;
  return L.off[level];
}
