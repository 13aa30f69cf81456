// gemm4s_kernel instantiations for epilogue ACT = 3 (see gemm4s.h)
#include "gemm4s.h"

namespace rtdc {
namespace g8 {
int gemm4s_launch_a3(const GemmArgs& a, const SkArgs& s, int a_kmajor, int b_kmajor, hipStream_t st) {
  return gemm4s_launch_act<3>(a, s, a_kmajor, b_kmajor, st);
}
}  // namespace g8
}  // namespace rtdc
