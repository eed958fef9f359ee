// gpad_panel.hip -- shared-matrix batches on the f32 MFMA pipe (placeholder until the panel
// kernel lands; reports "unsupported" so the runtime falls back to the row kernels).
#include <hip/hip_runtime.h>

#include "gpad_internal.h"

namespace gpad {
size_t panel_frag_bytes(int, int) { return 0; }
hipError_t launch_pack_panel(const float*, const float*, int, int, float, double, void*, hipStream_t) {
    return hipSuccess;
}
hipError_t launch_panel(const SolveArgs<float>&, hipStream_t, bool* supported) {
    *supported = false;
    return hipSuccess;
}
}  // namespace gpad
