// at_node.h -- transport-free core of the AprilTag node over include/at_api.h.
//
// The per-frame logic of the reference ROS 2 node ApriltagsDetector
// (src/apriltags_cuda/src/apriltags_cuda_detector.cu:7-605) with the ROS,
// cv_bridge, OpenCV and NetworkTables dependencies cut off at plain C++ types:
//   * parameters and defaults (setup_topics / setup_measurement_params, :93-133, :558-593);
//   * camera calibration from calibrationmatrix_<serial>.json (:315-371) and the
//     extrinsics from system_config.json (:196-300);
//   * imageCallback (:382-557): detect on the GPU (BGR8 goes straight in: no
//     cvtColor), GPU pose of every tag, transformCameraToRobot, sort by distance,
//     the two TagDetectionArray payloads (robot frame, camera frame), the
//     NetworkTables vector [t, id, x, y, z] * n, the ApriltagListProto bytes
//     (proto/apriltag.proto:6-17, AprilTagDataSender.cpp:32-39), the outlined
//     image (draw_detection_outlines, apriltag_utils.cu:54-79) and the
//     measurement CSV row.
// node/ros2_apriltags_node.cpp binds this core to rclcpp where ROS 2 exists;
// node/at_mock_node.cpp drives it from raw frame files (this image has no ROS 2).
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../include/at_api.h"

namespace at_node {

// Node parameters with the reference defaults (apriltags_cuda_detector.cu:93-133, :558-593).
struct Params {
  std::string topic_name = "camera/image_raw";
  std::string camera_serial = "N/A";
  std::string publish_images_to_topic = "apriltags/images";
  std::string publish_pose_to_topic = "camera/pose";
  int pin_to_core = -1;
  int priority = 80;
  bool measurement_mode = false;
  std::string timing_csv_path;  // "" -> apriltags_timing_YYYYMMDD_hhmmss.csv
};

// rclcpp::QoS(1).best_effort().durability_volatile().deadline(50 ms) of the subscription.
struct SubscriptionQos {
  int depth = 1;
  bool best_effort = true;
  bool volatile_durability = true;
  int deadline_ms = 50;
};

// apriltags_cuda/msg/TagDetection.msg: int32 id; float64 x, y, z.
struct TagDetectionMsg {
  int32_t id;
  double x, y, z;
};

// Everything one imageCallback publishes.
struct FrameOutputs {
  std::vector<at_detection> detections;           // id-sorted GPU detections
  std::vector<at_tag_detection> tags;             // closest first
  std::vector<TagDetectionMsg> robot;             // TagDetectionArray on <publish_pose_to_topic>
  std::vector<TagDetectionMsg> camera;            // ... on <publish_pose_to_topic>_camera
  std::vector<double> networktables_pose_data;    // [t, id, x, y, z] * n
  std::string proto;                              // serialized ApriltagListProto
  int status = AT_OK;                             // at_detect return code
  int64_t det_time_us = 0;
};

// calibrationmatrix_<serial>.json: "matrix" 3x3 and "disto" [[k1 k2 p1 p2 k3]].
bool load_camera_calibration(const std::string& dir, const std::string& serial, at_camera* cam, std::string* err);

// system_config.json: camera_mounted_positions[serial] (string, or {"location": ...})
// -> extrinsics[location].rotation (3x3) / offset (3).  Identity / zero and false when
// the camera or its location is missing (the reference logs and keeps its defaults).
bool load_extrinsics(const std::string& path, const std::string& serial, double R[9], double t[3],
                     std::string* location);

// ApriltagListProto{repeated ApriltagProto tags = 1} with ApriltagProto{collect_time = 1,
// tag_id = 2, x = 3, y = 4, z = 5} (proto2, all required), robot-frame coordinates in the
// order given (the node passes them closest first, :480-486).
std::string encode_apriltag_list(const at_tag_detection* tags, int n, double collect_time);

// Outline every detection on a bgr8 image in place (apriltag_utils.cu:54-79): p0-p1
// green, p0-p3 red, p1-p2 and p2-p3 blue, 2 px, and the id centred on c in (255,153,0).
// Line and glyph rasterization are this library's own (no OpenCV): the geometry and
// colours follow the reference, the exact pixels of cv::line / cv::putText do not.
void draw_detection_outlines(uint8_t* bgr, int width, int height, const at_detection* dets, int n);

class DetectorCore {
 public:
  // width/height of the camera frames; throws std::runtime_error when at_create fails.
  DetectorCore(int width, int height, const Params& params, const at_camera& cam, const double extr_R[9],
               const double extr_t[3], int device = 0);
  ~DetectorCore();
  DetectorCore(const DetectorCore&) = delete;
  DetectorCore& operator=(const DetectorCore&) = delete;

  // One frame (imageCallback): `frame` is bgr8 [H][W][3], yuyv [H][2W] or gray [H][W];
  // stamp_s = header.stamp, receive_s = node clock at receipt (latency column of the CSV).
  // `annotate` (bgr8 only, may be null) receives the outlined copy of the frame.
  int process(const uint8_t* frame, at_pixfmt fmt, double stamp_s, double receive_s, FrameOutputs* out,
              std::vector<uint8_t>* annotate = nullptr);

  const Params& params() const { return params_; }
  std::string pose_topic() const { return params_.publish_pose_to_topic; }
  std::string camera_pose_topic() const { return params_.publish_pose_to_topic + "_camera"; }
  const std::string& csv_path() const { return csv_path_; }

  // Publish hooks the transport binds (publish time lands in the CSV row).
  void (*publish_robot)(void* ctx, const std::vector<TagDetectionMsg>&) = nullptr;
  void (*publish_camera)(void* ctx, const std::vector<TagDetectionMsg>&) = nullptr;
  void (*publish_image)(void* ctx, const std::vector<uint8_t>&) = nullptr;
  void (*send_networktables)(void* ctx, const std::vector<double>&, const std::string& proto) = nullptr;
  void* ctx = nullptr;

 private:
  int width_, height_;
  Params params_;
  double R_[9], t_[3];
  at_detector* det_ = nullptr;
  std::vector<at_detection> dets_;
  std::vector<at_pose> poses_;
  std::FILE* csv_ = nullptr;
  std::string csv_path_;
};

}  // namespace at_node
