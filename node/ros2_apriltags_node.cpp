// ros2_apriltags_node.cpp -- ROS 2 binding of the node core (built by CMakeLists.txt only
// where rclcpp, sensor_msgs and the reference's apriltags_cuda messages exist; ROS 2 is not
// installed in this image, so this file is not compiled here).
//
// Drop-in for ApriltagsDetector (src/apriltags_cuda/src/apriltags_cuda_detector.cu): same
// parameters (topic_name, camera_serial, publish_images_to_topic, publish_pose_to_topic,
// pin_to_core, priority, measurement_mode, timing_csv_path), subscription QoS (depth 1,
// best effort, volatile, 50 ms deadline), TagDetectionArray publishers on <pose> (robot
// frame) and <pose>_camera, the outlined bgr8 image through a drop-oldest publisher
// queue.  Set-up as the reference's (apriltags_cuda_detector.cu:137-193, 601-605): frame
// W x H, intrinsics and extrinsics from the camera serial's records in
// vision_config_data's share directory (ament_index), then CPU pinning + SCHED_FIFO.
// The launch file (launch_vision.py:283-305) passes nothing else.
// The NetworkTables double array and ApriltagListProto are handed to the reference's
// AprilTagDataSender (wpilib) when the workspace provides it (send_networktables hook).
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "ament_index_cpp/get_package_share_directory.hpp"
#include "apriltags_cuda/msg/tag_detection.hpp"
#include "apriltags_cuda/msg/tag_detection_array.hpp"
#include "at_node.h"
#include "rclcpp/rclcpp.hpp"
#include "sensor_msgs/msg/image.hpp"

class ApriltagsAmdNode : public rclcpp::Node {
 public:
  ApriltagsAmdNode() : Node("apriltags_cuda_detector") {
    at_node::Params p;
    p.topic_name = declare_parameter<std::string>("topic_name", p.topic_name);
    p.camera_serial = declare_parameter<std::string>("camera_serial", p.camera_serial);
    p.publish_images_to_topic = declare_parameter<std::string>("publish_images_to_topic", p.publish_images_to_topic);
    p.publish_pose_to_topic = declare_parameter<std::string>("publish_pose_to_topic", p.publish_pose_to_topic);
    p.pin_to_core = declare_parameter<int>("pin_to_core", p.pin_to_core);
    p.priority = declare_parameter<int>("priority", p.priority);
    p.measurement_mode = declare_parameter<bool>("measurement_mode", p.measurement_mode);
    p.timing_csv_path = declare_parameter<std::string>("timing_csv_path", p.timing_csv_path);
    // optional override of the share directory (not passed by the launch file)
    std::string share_dir = declare_parameter<std::string>("vision_config_dir", "");
    if (share_dir.empty()) {
      try {
        share_dir = ament_index_cpp::get_package_share_directory("vision_config_data");
      } catch (const std::exception& e) {
        RCLCPP_ERROR(get_logger(), "vision_config_data: %s", e.what());
      }
    }
    at_node::NodeConfig config;
    std::string err;
    if (!at_node::resolve_node_config(p.camera_serial, share_dir, &config, &err)) {
      RCLCPP_ERROR(get_logger(), "%s", err.c_str());
      throw std::runtime_error(err);  // as setup_apriltags (:162-169)
    }
    if (!config.have_extrinsics)
      RCLCPP_ERROR(get_logger(), "no extrinsics for camera %s: identity / zero", p.camera_serial.c_str());
    RCLCPP_INFO(get_logger(), "Using camera config dimensions: %dx%d for serial %s", config.camera.width,
                config.camera.height, p.camera_serial.c_str());
    const int width = config.camera.width, height = config.camera.height;
    core_ = std::make_unique<at_node::DetectorCore>(p, config);
    core_->ctx = this;
    core_->publish_robot = [](void* c, const std::vector<at_node::TagDetectionMsg>& v) {
      static_cast<ApriltagsAmdNode*>(c)->pose_pub_->publish(to_msg(v));
    };
    core_->publish_camera = [](void* c, const std::vector<at_node::TagDetectionMsg>& v) {
      static_cast<ApriltagsAmdNode*>(c)->camera_pose_pub_->publish(to_msg(v));
    };
    core_->publish_image = [](void* c, const std::vector<uint8_t>& bgr, double stamp_s) {
      auto* self = static_cast<ApriltagsAmdNode*>(c);  // publisher-queue thread
      auto msg = std::make_unique<sensor_msgs::msg::Image>();
      msg->header.stamp = rclcpp::Time(static_cast<int64_t>(stamp_s * 1e9));  // image_capture_time (:516)
      msg->header.frame_id = "apriltag_detections";
      msg->width = self->width_;
      msg->height = self->height_;
      msg->encoding = "bgr8";
      msg->step = self->width_ * 3;
      msg->data = bgr;
      self->image_pub_->publish(std::move(msg));
    };
    width_ = width;
    height_ = height;
    auto qos = rclcpp::QoS(1).best_effort().durability_volatile().deadline(std::chrono::milliseconds(50));
    sub_ = create_subscription<sensor_msgs::msg::Image>(
        p.topic_name, qos, [this](sensor_msgs::msg::Image::SharedPtr m) { on_image(m); });
    pose_pub_ = create_publisher<apriltags_cuda::msg::TagDetectionArray>(p.publish_pose_to_topic, 10);
    camera_pose_pub_ = create_publisher<apriltags_cuda::msg::TagDetectionArray>(core_->camera_pose_topic(), 10);
    image_pub_ = create_publisher<sensor_msgs::msg::Image>(p.publish_images_to_topic, 10);
    std::string sched_log;  // applyCpuPinningAndScheduling (:601-605)
    at_node::apply_cpu_pinning_and_scheduling(p.pin_to_core, p.priority, &sched_log);
    RCLCPP_INFO(get_logger(), "%s", sched_log.c_str());
  }

 // Teardown order: no more image callbacks, then the publisher-queue thread drained
  // and joined while image_pub_ is still alive (its publish hook uses it), then the
  // detector; only then the publishers (declared before core_, so destroyed after it).
  ~ApriltagsAmdNode() override {
    sub_.reset();
    if (core_) core_->flush_images();
    core_.reset();
  }

 private:
  static apriltags_cuda::msg::TagDetectionArray to_msg(const std::vector<at_node::TagDetectionMsg>& v) {
    apriltags_cuda::msg::TagDetectionArray a;
    for (const auto& d : v) {
      apriltags_cuda::msg::TagDetection t;
      t.id = d.id;
      t.x = d.x;
      t.y = d.y;
      t.z = d.z;
      a.detections.push_back(t);
    }
    return a;
  }

  void on_image(const sensor_msgs::msg::Image::SharedPtr& m) {
    if ((int)m->width != width_ || (int)m->height != height_) {
      RCLCPP_ERROR(get_logger(), "frame %ux%u, detector %dx%d", m->width, m->height, width_, height_);
      return;
    }
    at_pixfmt fmt;
    size_t row;
    if (m->encoding == "bgr8") { fmt = AT_FMT_BGR8; row = 3 * (size_t)width_; }
    else if (m->encoding == "yuv422_yuy2" || m->encoding == "yuyv") { fmt = AT_FMT_YUYV; row = 2 * (size_t)width_; }
    else if (m->encoding == "mono8") { fmt = AT_FMT_GRAY8; row = width_; }
    else {
      RCLCPP_ERROR(get_logger(), "unsupported encoding %s", m->encoding.c_str());
      return;
    }
    const uint8_t* frame = m->data.data();
    if (m->step != row) {  // padded rows: pack them (the detector takes dense frames)
      packed_.resize(row * height_);
      for (int y = 0; y < height_; ++y) std::memcpy(packed_.data() + row * y, m->data.data() + (size_t)m->step * y, row);
      frame = packed_.data();
    }
    const double stamp = rclcpp::Time(m->header.stamp).seconds();
    at_node::FrameOutputs out;
    const int rc = core_->process(frame, fmt, stamp, now().seconds(), &out, fmt == AT_FMT_BGR8 ? &image_ : nullptr);
    if (rc != AT_OK) RCLCPP_WARN(get_logger(), "at_detect: %s", at_strerror(rc));
  }

  int width_ = 0, height_ = 0;
  std::vector<uint8_t> packed_;
  at_node::ImageBuffer image_;  // page-locked: the annotated image arrives by DMA
  rclcpp::Publisher<apriltags_cuda::msg::TagDetectionArray>::SharedPtr pose_pub_, camera_pose_pub_;
  rclcpp::Publisher<sensor_msgs::msg::Image>::SharedPtr image_pub_;
  // after the publishers: destroyed first (members go in reverse order), so the
  // publisher-queue thread never outlives image_pub_
  std::unique_ptr<at_node::DetectorCore> core_;
  rclcpp::Subscription<sensor_msgs::msg::Image>::SharedPtr sub_;
};

int main(int argc, char** argv) {
  rclcpp::init(argc, argv);
  rclcpp::spin(std::make_shared<ApriltagsAmdNode>());
  rclcpp::shutdown();
  return 0;
}
