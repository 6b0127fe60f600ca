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

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../include/at_api.h"

namespace at_node {

// Page-locked allocation (at_host_alloc) for the annotated image: at_annotate_staged
// then copies it out of HBM by DMA on the detector's stream instead of through the
// runtime's staging of a pageable destination.
template <class T>
struct PinnedAllocator {
  using value_type = T;
  PinnedAllocator() = default;
  template <class U>
  PinnedAllocator(const PinnedAllocator<U>&) {}
  T* allocate(size_t n) {
    void* p = nullptr;
    if (at_host_alloc(n * sizeof(T), &p) != AT_OK || !p) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t) { at_host_free(p); }
  template <class U>
  bool operator==(const PinnedAllocator<U>&) const { return true; }
  template <class U>
  bool operator!=(const PinnedAllocator<U>&) const { return false; }
};
using ImageBuffer = std::vector<uint8_t, PinnedAllocator<uint8_t>>;

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

// ---- vision_config_data / vision_utils::ConfigLoader -------------------------
// One camera record of system_config.json camera_mounted_positions
// (vision_utils/config_loader.cpp:77-105): a record is used only when every field
// below is present with its type (integers for width / height / frame_rate).
struct CameraConfig {
  std::string location = "center_front", format = "MJPG", api_preference = "V4L2";
  int height = 800, width = 1280, frame_rate = 100;
};
struct NetworkTablesConfig {  // config_loader.hpp defaults, :143-152 of the .cpp
  std::string table_address = "10.7.66.2", table_name = "/SmartDashboard";
};
// ament_index_cpp::get_package_share_directory over $AMENT_PREFIX_PATH: the first
// prefix holding share/ament_index/resource_index/packages/<package> gives
// <prefix>/share/<package>; "" when no prefix has it.
std::string package_share_directory(const std::string& package);
// ConfigLoader::getCameraConfig (config_loader.cpp:158-170): false when the file is
// unreadable or the serial has no complete record.
bool load_camera_config(const std::string& system_config_path, const std::string& serial, CameraConfig* out);
NetworkTablesConfig load_network_tables_config(const std::string& system_config_path);

// Everything ApriltagsDetector::setup_apriltags derives from the camera serial
// (apriltags_cuda_detector.cu:137-193, 203-301, 315-371), from the vision_config_data
// share directory: W x H from the camera record (required: the reference throws),
// intrinsics from data/calibration/calibrationmatrix_<serial>.json (required),
// extrinsics from data/system_config.json (optional: identity / zero, as the
// reference keeps its defaults), the NetworkTables address.
struct NodeConfig {
  std::string share_dir, system_config, calibration_dir, location;
  CameraConfig camera;
  NetworkTablesConfig networktables;
  at_camera cam{};
  double R[9], t[3];
  bool have_extrinsics = false;
};
// share_dir "" resolves vision_config_data through $AMENT_PREFIX_PATH.
bool resolve_node_config(const std::string& serial, const std::string& share_dir, NodeConfig* out, std::string* err);

// vision_utils::ProcessScheduler::applyCpuPinningAndScheduling (process_scheduler.cpp:23-50)
// for the calling thread: pin_to_core == -1 does nothing; otherwise affinity to that
// core (0 <= core < online CPUs) and SCHED_FIFO at `priority`, both attempted, then
// verified.  false if either failed (e.g. no CAP_SYS_NICE); `log` gets the messages.
bool apply_cpu_pinning_and_scheduling(int pin_to_core, int priority, std::string* log);

// vision_utils PublisherQueue (publisher_queue.hpp:10-65): a worker thread publishes
// what enqueue() hands it; the queue keeps at most max_size entries and drops the
// oldest when full, so a slow subscriber never stalls the image callback.
template <typename T>
class PublisherQueue {
 public:
  PublisherQueue(std::function<void(const T&)> publish, size_t max_size = 2)
      : publish_(std::move(publish)), max_(max_size), running_(true), thread_(&PublisherQueue::run, this) {}
  ~PublisherQueue() { stop(); }
  void enqueue(T msg) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (q_.size() >= max_) {
        q_.pop_front();
        ++dropped_;
      }
      q_.push_back(std::move(msg));
    }
    cv_.notify_one();
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      running_ = false;
    }
    cv_.notify_all();
    if (thread_.joinable()) thread_.join();
  }
  size_t dropped() const { return dropped_; }

 private:
  void run() {
    for (;;) {
      T msg;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty() || !running_; });
        if (q_.empty()) return;  // stopped and drained
        msg = std::move(q_.front());
        q_.pop_front();
      }
      publish_(msg);
    }
  }
  std::function<void(const T&)> publish_;
  size_t max_;
  std::deque<T> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool running_;
  std::atomic<size_t> dropped_{0};
  std::thread thread_;
};

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
  // The reference node's set-up: W x H, intrinsics and extrinsics from the camera
  // serial's records (resolve_node_config).
  DetectorCore(const Params& params, const NodeConfig& config, int device = 0);
  ~DetectorCore();
  DetectorCore(const DetectorCore&) = delete;
  DetectorCore& operator=(const DetectorCore&) = delete;

  // One frame (imageCallback): `frame` is bgr8 [H][W][3], yuyv [H][2W] or gray [H][W];
  // stamp_s = header.stamp, receive_s = node clock at receipt (latency column of the CSV).
  // `annotate` (bgr8 only, may be null) receives the outlined copy of the frame, drawn
  // on the GPU on the frame already staged in HBM (at_annotate_staged); publish_image
  // then gets it from the drop-oldest PublisherQueue thread (depth 2, :50-52, :518).
  int process(const uint8_t* frame, at_pixfmt fmt, double stamp_s, double receive_s, FrameOutputs* out,
              ImageBuffer* annotate = nullptr);

  const Params& params() const { return params_; }
  int width() const { return width_; }
  int height() const { return height_; }
  // images the publisher queue dropped (a subscriber slower than the frame rate)
  size_t images_dropped() const { return image_queue_ ? image_queue_->dropped() : 0; }
  // waits until the publisher queue has handed every queued image to publish_image
  void flush_images() { image_queue_.reset(); }
  std::string pose_topic() const { return params_.publish_pose_to_topic; }
  std::string camera_pose_topic() const { return params_.publish_pose_to_topic + "_camera"; }
  const std::string& csv_path() const { return csv_path_; }

  // Publish hooks the transport binds (publish time lands in the CSV row).
  void (*publish_robot)(void* ctx, const std::vector<TagDetectionMsg>&) = nullptr;
  void (*publish_camera)(void* ctx, const std::vector<TagDetectionMsg>&) = nullptr;
  // called on the publisher-queue thread with the annotated image and its frame's stamp
  void (*publish_image)(void* ctx, const std::vector<uint8_t>&, double stamp_s) = nullptr;
  void (*send_networktables)(void* ctx, const std::vector<double>&, const std::string& proto) = nullptr;
  void* ctx = nullptr;

 private:
  void init(const at_camera& cam, int device);
  int width_, height_;
  Params params_;
  struct StampedImage {
    std::vector<uint8_t> bgr;
    double stamp_s = 0;
  };
  std::unique_ptr<PublisherQueue<StampedImage>> image_queue_;
  double R_[9], t_[3];
  at_detector* det_ = nullptr;
  std::vector<at_detection> dets_;
  std::vector<at_pose> poses_;
  std::FILE* csv_ = nullptr;
  std::string csv_path_;
};

}  // namespace at_node
