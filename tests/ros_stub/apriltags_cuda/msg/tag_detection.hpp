// Type-check stand-in of the reference's msg/TagDetection.msg (see ../../README.md).
#pragma once
#include <cstdint>
namespace apriltags_cuda::msg {
struct TagDetection {
  int32_t id = 0;
  double x = 0, y = 0, z = 0;
};
}  // namespace apriltags_cuda::msg
