// fa_windowed.hip — windowed attention (placeholder until the fused kernel lands).
#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"
namespace fa {
size_t windowed_workspace(int, const WindowGeom&, int64_t, int64_t, int64_t) { return 0; }
int launch_windowed_fwd(const WindowedArgs&, hipStream_t, const char** why) {
    *why = "windowed forward not built yet";
    return FA_ERR_UNSUPPORTED;
}
int launch_windowed_bwd(const WindowedBwdArgs&, hipStream_t, const char** why) {
    *why = "windowed backward not built yet";
    return FA_ERR_UNSUPPORTED;
}
}  // namespace fa
