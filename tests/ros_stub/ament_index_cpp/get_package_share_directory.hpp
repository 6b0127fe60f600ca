// Type-check stand-in (see ../README.md).
#pragma once
#include <string>
namespace ament_index_cpp {
inline std::string get_package_share_directory(const std::string& p) { return p; }
}  // namespace ament_index_cpp
