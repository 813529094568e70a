// Error helpers for a tools-only build of one kernel file (tools/ab_attn.sh): the product
// definitions live in csrc/elementwise.hip.
#include <hip/hip_runtime.h>
#include <string>
namespace vc {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
int fail(int code, const std::string& m) { g_err = m; return code; }
int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { g_err = std::string(what) + ": " + hipGetErrorString(e); return (int)e; }
    return 0;
}
}  // namespace vc
