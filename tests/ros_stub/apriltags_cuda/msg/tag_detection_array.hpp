// Type-check stand-in of the reference's msg/TagDetectionArray.msg (see ../../README.md).
#pragma once
#include <vector>
#include "apriltags_cuda/msg/tag_detection.hpp"
namespace apriltags_cuda::msg {
struct TagDetectionArray {
  std::vector<TagDetection> detections;
};
}  // namespace apriltags_cuda::msg
