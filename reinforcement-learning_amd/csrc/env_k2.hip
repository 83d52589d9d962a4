// env_k2.hip -- the env kernel specialised for RLGPU_ARITH_SCALAR (env_step.hpp), its constant uploads and its launch.
#define RLGPU_ENV_ARITH 2
#define RLGPU_ENV_KERNEL env_kernel_a2
#include "common.hpp"
#include "env_step.hpp"

namespace rl {
void env_k2_upload(const EnvConst& k, const RsqrtLut* lut) {
    RLGPU_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(C), &k, sizeof k));
    if (lut) RLGPU_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kRsqrtLut), lut, sizeof *lut));
}
void env_k2_launch(const StepArgs& g, int blocks, hipStream_t s) {
    hipLaunchKernelGGL(env_kernel_a2, dim3(blocks), dim3(kWG), 0, s, g);
    RLGPU_CHECK_HIP(hipGetLastError());
}
}  // namespace rl
