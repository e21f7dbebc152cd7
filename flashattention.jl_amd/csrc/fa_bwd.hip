// fa_bwd.hip — dense backward (placeholder until the MFMA kernel lands).
#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"
namespace fa {
size_t dense_bwd_workspace(int, int64_t, int64_t, int64_t, int64_t, int64_t) { return 0; }
int launch_dense_bwd(const DenseBwdArgs&, hipStream_t, const char** why) {
    *why = "backward not built yet";
    return FA_ERR_UNSUPPORTED;
}
}  // namespace fa
