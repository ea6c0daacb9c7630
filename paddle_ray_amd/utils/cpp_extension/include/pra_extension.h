// paddle_ray_amd custom-operator ABI (the role of paddle/extension.h + PD_BUILD_OP in the
// reference, python/paddle/utils/cpp_extension). A custom op is plain C/C++ or HIP code that
// sees tensors as PraTensor views (device pointer, shape, dtype) and the caller's HIP stream;
// it never links against the framework. utils.cpp_extension.load() compiles the sources
// (g++ for .cc/.cpp, hipcc --offload-arch=gfx950 for .hip), loads the library and wraps every
// registered op as a Python function with autograd (its backward kernel) and a kernel-registry
// entry.
//
//   static int relu_infer(const PraTensor* in, int nin, PraTensor* out, int nout) {
//     out[0] = in[0];                 // same shape / dtype as the input (data is ignored)
//     return 0;
//   }
//   static int relu_fwd(const PraTensor* in, int nin, PraTensor* out, int nout, void* stream);
//   static int relu_bwd(const PraTensor* in, int nin, PraTensor* out, int nout, void* stream);
//   PRA_REGISTER_OP(custom_relu, 1, 1, relu_fwd, relu_infer, relu_bwd)
//
// forward:  in = the op inputs, out = its outputs (allocated by the framework from infer).
// backward: in = [forward inputs..., forward outputs..., output gradients...],
//           out = the input gradients (allocated like the inputs). nullptr = no gradient.
// Return 0 on success; non-zero raises in Python. Tensors are contiguous row-major.
#pragma once
#include <stdint.h>
#include <vector>

#define PRA_MAX_DIMS 8

enum PraDType : int32_t {
  PRA_F32 = 0, PRA_F16 = 1, PRA_BF16 = 2, PRA_F64 = 3, PRA_I32 = 4, PRA_I64 = 5, PRA_U8 = 6, PRA_BOOL = 7
};

extern "C" {
typedef struct PraTensor {
  void* data;
  int64_t numel;
  int32_t ndim;
  int32_t dtype;  // PraDType
  int64_t shape[PRA_MAX_DIMS];
} PraTensor;

typedef int (*PraOpFn)(const PraTensor* in, int n_in, PraTensor* out, int n_out, void* stream);
typedef int (*PraInferFn)(const PraTensor* in, int n_in, PraTensor* out, int n_out);

typedef struct PraOpDef {
  const char* name;
  int n_in, n_out;
  PraOpFn forward;
  PraInferFn infer;
  PraOpFn backward;
} PraOpDef;
}

namespace pra_ext {
inline std::vector<PraOpDef>& registry() {
  static std::vector<PraOpDef> ops;
  return ops;
}
struct Registrar {
  explicit Registrar(PraOpDef d) { registry().push_back(d); }
};
inline int64_t numel_of(const PraTensor& t) {
  int64_t n = 1;
  for (int i = 0; i < t.ndim; ++i) n *= t.shape[i];
  return n;
}
}  // namespace pra_ext

// the library's op table (weak: every translation unit that includes this header emits it,
// the linker keeps one)
extern "C" __attribute__((weak, visibility("default"))) int pra_ext_num_ops() {
  return (int)pra_ext::registry().size();
}
extern "C" __attribute__((weak, visibility("default"))) const PraOpDef* pra_ext_op(int i) {
  return &pra_ext::registry()[i];
}

#define PRA_REGISTER_OP(NAME, NIN, NOUT, FWD, INFER, BWD) \
  static pra_ext::Registrar pra_ext_reg_##NAME(PraOpDef{#NAME, NIN, NOUT, FWD, INFER, BWD});
