// C-ABI housekeeping for libxtrl_hip: version and the per-thread last-error message.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/xtrl_hip.h"
#include "philox.h"

namespace xtrl {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return XTRL_E_HIP;
  }
  return XTRL_OK;
}

}  // namespace xtrl

extern "C" int xtrl_abi_version(void) { return XTRL_ABI_VERSION; }

#ifndef XTRL_SRC_HASH
#define XTRL_SRC_HASH "unknown"
#endif
// content hash of the sources this library was compiled from (xtrl_amd/_srchash.py)
extern "C" const char* xtrl_source_hash(void) { return XTRL_SRC_HASH; }

// sizeof of a descriptor struct as compiled into the library (bindings check their mirrors)
extern "C" int64_t xtrl_struct_size(const char* name) {
  static const struct {
    const char* name;
    int64_t size;
  } sizes[] = {{"XtrlDecodeLayer", sizeof(XtrlDecodeLayer)}, {"XtrlRngState", sizeof(XtrlRngState)},
               {"XtrlDecodeDesc", sizeof(XtrlDecodeDesc)},   {"XtrlTrainLayer", sizeof(XtrlTrainLayer)},
               {"XtrlTrainDesc", sizeof(XtrlTrainDesc)},     {"XtrlBatchDesc", sizeof(XtrlBatchDesc)},
               {"XtrlLossDesc", sizeof(XtrlLossDesc)},       {"XtrlFractalLevel", sizeof(XtrlFractalLevel)},
               {"XtrlFractalDesc", sizeof(XtrlFractalDesc)},     {"XtrlFractalTrainLevel", sizeof(XtrlFractalTrainLevel)},
               {"XtrlFractalTrainDesc", sizeof(XtrlFractalTrainDesc)}};
  for (const auto& s : sizes)
    if (name && strcmp(name, s.name) == 0) return s.size;
  return -1;
}
extern "C" const char* xtrl_last_error(void) { return xtrl::g_err; }

// host-side views of the device random streams (reward-dropout coin, tests)
extern "C" float xtrl_rng_uniform(uint64_t seed, uint32_t update, uint32_t slot, uint32_t t, uint32_t field,
                                  uint32_t sub) {
  return xtrl::rng_uniform(seed, update, slot, t, field, sub);
}
extern "C" float xtrl_rng_normal(uint64_t seed, uint32_t update, uint32_t slot, uint32_t t, uint32_t field,
                                 uint32_t sub) {
  return xtrl::rng_normal(seed, update, slot, t, field, sub);
}
