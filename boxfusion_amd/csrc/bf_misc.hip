// bf_misc.hip — library identity
#include "bf_common.h"

BF_API const char* bf_version(void) { return "boxfusion_hip 0.1.0 gfx950"; }

BF_API int bf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
