// gfx950 custom op for tests/test_cpp_extension.py: the same custom_relu on the device, bf16 or
// fp32, one element per lane, launched on the caller's HIP stream
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include "pra_extension.h"

template <typename T>
__global__ void relu_k(const T* x, T* y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (float)x[i] > 0.f ? x[i] : T(0.f);
}
template <typename T>
__global__ void relu_bwd_k(const T* x, const T* dy, T* dx, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = (float)x[i] > 0.f ? dy[i] : T(0.f);
}

static int relu_infer(const PraTensor* in, int, PraTensor* out, int) {
  out[0] = in[0];
  return 0;
}
static int relu_fwd(const PraTensor* in, int, PraTensor* out, int, void* s) {
  const int64_t n = in[0].numel;
  const int blocks = (int)((n + 255) / 256);
  if (n == 0) return 0;
  if (in[0].dtype == PRA_F32)
    relu_k<float><<<blocks, 256, 0, (hipStream_t)s>>>((const float*)in[0].data, (float*)out[0].data, n);
  else if (in[0].dtype == PRA_BF16)
    relu_k<__hip_bfloat16><<<blocks, 256, 0, (hipStream_t)s>>>((const __hip_bfloat16*)in[0].data,
                                                               (__hip_bfloat16*)out[0].data, n);
  else
    return 1;
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
static int relu_bwd(const PraTensor* in, int, PraTensor* out, int, void* s) {
  const int64_t n = in[0].numel;
  const int blocks = (int)((n + 255) / 256);
  if (n == 0) return 0;
  if (in[0].dtype == PRA_F32)
    relu_bwd_k<float><<<blocks, 256, 0, (hipStream_t)s>>>((const float*)in[0].data, (const float*)in[2].data,
                                                          (float*)out[0].data, n);
  else if (in[0].dtype == PRA_BF16)
    relu_bwd_k<__hip_bfloat16><<<blocks, 256, 0, (hipStream_t)s>>>(
        (const __hip_bfloat16*)in[0].data, (const __hip_bfloat16*)in[2].data, (__hip_bfloat16*)out[0].data, n);
  else
    return 1;
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

PRA_REGISTER_OP(custom_relu, 1, 1, relu_fwd, relu_infer, relu_bwd)
