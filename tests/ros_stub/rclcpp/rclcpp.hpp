// Type-check stand-in of the rclcpp API surface the node binding uses (see ../README.md).
#pragma once
#include <chrono>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>

#include "builtin_interfaces/msg/time.hpp"

namespace rclcpp {
struct Logger {};
struct Time {
  Time() = default;
  explicit Time(int64_t) {}
  Time(const builtin_interfaces::msg::Time&) {}  // NOLINT: implicit like rclcpp
  double seconds() const { return 0; }
  operator builtin_interfaces::msg::Time() const { return {}; }
};
struct QoS {
  explicit QoS(size_t) {}
  QoS& best_effort() { return *this; }
  QoS& durability_volatile() { return *this; }
  template <class R, class P>
  QoS& deadline(std::chrono::duration<R, P>) { return *this; }
};
template <class M>
struct Subscription {
  using SharedPtr = std::shared_ptr<Subscription>;
};
template <class M>
struct Publisher {
  using SharedPtr = std::shared_ptr<Publisher>;
  void publish(const M&) {}
  void publish(std::unique_ptr<M>) {}
};
class Node {
 public:
  explicit Node(const std::string&) {}
  virtual ~Node() = default;
  template <class T>
  T declare_parameter(const std::string&, const T& v) { return v; }
  Logger get_logger() const { return {}; }
  Time now() const { return Time(); }
  template <class M, class F>
  typename Subscription<M>::SharedPtr create_subscription(const std::string&, const QoS&, F&&) { return nullptr; }
  template <class M>
  typename Publisher<M>::SharedPtr create_publisher(const std::string&, size_t) { return nullptr; }
};
inline void init(int, char**) {}
inline void spin(std::shared_ptr<Node>) {}
inline void shutdown() {}
}  // namespace rclcpp

#define RCLCPP_INFO(logger, ...) ((void)(logger), (void)sizeof(printf(__VA_ARGS__)))
#define RCLCPP_WARN(logger, ...) ((void)(logger), (void)sizeof(printf(__VA_ARGS__)))
#define RCLCPP_ERROR(logger, ...) ((void)(logger), (void)sizeof(printf(__VA_ARGS__)))
