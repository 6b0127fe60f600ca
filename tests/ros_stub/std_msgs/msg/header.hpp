// Type-check stand-in (see ../../README.md).
#pragma once
#include <string>
#include "builtin_interfaces/msg/time.hpp"
namespace std_msgs::msg {
struct Header {
  builtin_interfaces::msg::Time stamp;
  std::string frame_id;
};
}  // namespace std_msgs::msg
