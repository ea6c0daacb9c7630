// host custom op for tests/test_cpp_extension.py: y = relu(x) * alpha-free, dx = dy * (x > 0)
#include "pra_extension.h"

static int relu_infer(const PraTensor* in, int, PraTensor* out, int) {
  out[0] = in[0];
  return 0;
}

static int relu_fwd(const PraTensor* in, int, PraTensor* out, int, void*) {
  if (in[0].dtype != PRA_F32) return 1;
  const float* x = static_cast<const float*>(in[0].data);
  float* y = static_cast<float*>(out[0].data);
  for (int64_t i = 0; i < in[0].numel; ++i) y[i] = x[i] > 0.f ? x[i] : 0.f;
  return 0;
}

// in = [x, y, dy], out = [dx]
static int relu_bwd(const PraTensor* in, int, PraTensor* out, int, void*) {
  const float* x = static_cast<const float*>(in[0].data);
  const float* dy = static_cast<const float*>(in[2].data);
  float* dx = static_cast<float*>(out[0].data);
  for (int64_t i = 0; i < in[0].numel; ++i) dx[i] = x[i] > 0.f ? dy[i] : 0.f;
  return 0;
}

// a two-input, two-output op: (a*b, a+b)
static int mul_add_infer(const PraTensor* in, int, PraTensor* out, int) {
  out[0] = in[0];
  out[1] = in[0];
  return 0;
}
static int mul_add_fwd(const PraTensor* in, int, PraTensor* out, int, void*) {
  const float* a = static_cast<const float*>(in[0].data);
  const float* b = static_cast<const float*>(in[1].data);
  float* p = static_cast<float*>(out[0].data);
  float* s = static_cast<float*>(out[1].data);
  for (int64_t i = 0; i < in[0].numel; ++i) { p[i] = a[i] * b[i]; s[i] = a[i] + b[i]; }
  return 0;
}
// in = [a, b, p, s, dp, ds], out = [da, db]
static int mul_add_bwd(const PraTensor* in, int, PraTensor* out, int, void*) {
  const float* a = static_cast<const float*>(in[0].data);
  const float* b = static_cast<const float*>(in[1].data);
  const float* dp = static_cast<const float*>(in[4].data);
  const float* ds = static_cast<const float*>(in[5].data);
  float* da = static_cast<float*>(out[0].data);
  float* db = static_cast<float*>(out[1].data);
  for (int64_t i = 0; i < in[0].numel; ++i) { da[i] = dp[i] * b[i] + ds[i]; db[i] = dp[i] * a[i] + ds[i]; }
  return 0;
}

PRA_REGISTER_OP(custom_relu, 1, 1, relu_fwd, relu_infer, relu_bwd)
PRA_REGISTER_OP(custom_mul_add, 2, 2, mul_add_fwd, mul_add_infer, mul_add_bwd)
