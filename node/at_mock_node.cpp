// at_mock_node.cpp -- the node core driven from raw frame files (no ROS 2 here).
//
// Stands in for the subscription: every frame of --frames (back-to-back raw
// bgr8 / yuyv / gray frames) is handed to DetectorCore::process exactly as
// ApriltagsDetector::imageCallback hands its cv_bridge image to the detector
// (apriltags_cuda_detector.cu:382-557).  Publishers print one JSON line per
// frame; --proto-out / --image-out write the ApriltagListProto bytes and the
// outlined bgr8 image of the last frame.
//
// usage: at_mock_node --camera-serial S --format bgr8|yuyv|gray --frames F [--count N]
//        [--vision-config-dir D] [--pin-to-core C --priority P]
//        [--measurement-csv PATH] [--proto-out P] [--image-out I] [--device K] [--time N]
//   As the reference node (apriltags_cuda_detector.cu:137-193): the frame size, the
//   intrinsics and the extrinsics come from the camera serial's records in the
//   vision_config_data share directory, found through $AMENT_PREFIX_PATH
//   (ament_index) or given with --vision-config-dir.  Without a serial's records
//   (test setups) --width W --height H [--calibration-dir D] [--system-config C]
//   give them directly (calibration default: the reference test camera).
//   --time N: after one untimed pass, N calls of DetectorCore::process over the frames
//   in turn (the whole callback: detect, poses, robot frame, messages, proto and, for
//   bgr8, the outlined image drawn on the GPU and copied out), one JSON line with the
//   p50 / p99 wall time per call instead of the per-frame lines.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "at_node.h"

namespace {
struct Sink {
  std::string robot, camera;
};
std::string msgs_json(const std::vector<at_node::TagDetectionMsg>& v) {
  std::string s = "[";
  char buf[160];
  for (size_t i = 0; i < v.size(); ++i) {
    std::snprintf(buf, sizeof(buf), "%s[%d,%.17g,%.17g,%.17g]", i ? "," : "", v[i].id, v[i].x, v[i].y, v[i].z);
    s += buf;
  }
  return s + "]";
}
void on_robot(void* ctx, const std::vector<at_node::TagDetectionMsg>& v) { ((Sink*)ctx)->robot = msgs_json(v); }
void on_camera(void* ctx, const std::vector<at_node::TagDetectionMsg>& v) { ((Sink*)ctx)->camera = msgs_json(v); }
}  // namespace

int main(int argc, char** argv) {
  int W = 0, H = 0, count = -1, device = 0, pin = -1, priority = 80, time_n = 0;
  std::string fmt_s = "yuyv", frames_path, calib_dir, serial = "N/A", sys_cfg, csv, proto_out, image_out, share_dir;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i], v = argv[i + 1];
    if (k == "--width") W = std::atoi(v.c_str());
    else if (k == "--height") H = std::atoi(v.c_str());
    else if (k == "--format") fmt_s = v;
    else if (k == "--frames") frames_path = v;
    else if (k == "--count") count = std::atoi(v.c_str());
    else if (k == "--calibration-dir") calib_dir = v;
    else if (k == "--camera-serial") serial = v;
    else if (k == "--system-config") sys_cfg = v;
    else if (k == "--measurement-csv") csv = v;
    else if (k == "--proto-out") proto_out = v;
    else if (k == "--image-out") image_out = v;
    else if (k == "--device") device = std::atoi(v.c_str());
    else if (k == "--vision-config-dir") share_dir = v;
    else if (k == "--pin-to-core") pin = std::atoi(v.c_str());
    else if (k == "--priority") priority = std::atoi(v.c_str());
    else if (k == "--time") time_n = std::atoi(v.c_str());
    else { std::fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
  }
  at_node::Params prm;
  prm.camera_serial = serial;
  prm.measurement_mode = !csv.empty();
  prm.timing_csv_path = csv;
  prm.pin_to_core = pin;
  prm.priority = priority;
  // the reference test camera (test/gpu_detector_test.cu:62-73) unless a calibration is given
  at_node::NodeConfig nc;
  nc.cam = at_camera{905.495617, 907.909470, 609.916016, 352.682645, 0.059238, -0.075154, -0.003801, 0.001113, 0.0};
  std::string err;
  if (W <= 0 && H <= 0) {  // the node's set-up: everything from the serial's records
    if (!at_node::resolve_node_config(serial, share_dir, &nc, &err)) {
      std::fprintf(stderr, "config: %s\n", err.c_str());
      return 1;
    }
  } else {
    nc.camera.width = W;
    nc.camera.height = H;
    if (!calib_dir.empty() && !at_node::load_camera_calibration(calib_dir, serial, &nc.cam, &err)) {
      std::fprintf(stderr, "calibration: %s\n", err.c_str());
      return 1;
    }
    at_node::load_extrinsics(sys_cfg.empty() ? "/nonexistent" : sys_cfg, serial, nc.R, nc.t, &nc.location);
  }
  W = nc.camera.width;
  H = nc.camera.height;
  const std::string& location = nc.location;
  const at_pixfmt fmt = fmt_s == "bgr8" ? AT_FMT_BGR8 : (fmt_s == "gray" ? AT_FMT_GRAY8 : AT_FMT_YUYV);
  const size_t fb = (size_t)W * H * (fmt == AT_FMT_BGR8 ? 3 : (fmt == AT_FMT_YUYV ? 2 : 1));
  if (W <= 0 || H <= 0 || frames_path.empty()) {
    std::fprintf(stderr, "usage: %s --camera-serial S --format bgr8|yuyv|gray --frames FILE ...\n", argv[0]);
    return 2;
  }
  std::ifstream in(frames_path, std::ios::binary);
  std::vector<uint8_t> all((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  const int nframes = (int)(all.size() / fb);
  if (count < 0 || count > nframes) count = nframes;
  if (time_n > 0 && count <= 0) {  // the timed loop walks the frames modulo count
    std::fprintf(stderr, "%s: --time needs at least one frame (--count %d, %d frames in %s)\n", argv[0], count,
                 nframes, frames_path.c_str());
    return 2;
  }
  // applyCpuPinningAndScheduling (:601-605): failures are logged, not fatal
  std::string sched_log;
  const bool sched_ok = at_node::apply_cpu_pinning_and_scheduling(prm.pin_to_core, prm.priority, &sched_log);
  std::fprintf(stderr, "%s", sched_log.c_str());
  std::printf("{\"width\":%d,\"height\":%d,\"fx\":%.17g,\"location\":\"%s\",\"scheduling_applied\":%s,"
              "\"networktables\":\"%s\"}\n",
              W, H, nc.cam.fx, location.c_str(), sched_ok ? "true" : "false", nc.networktables.table_address.c_str());
  Sink sink;
  try {
    at_node::DetectorCore core(prm, nc, device);
    core.publish_robot = on_robot;
    core.publish_camera = on_camera;
    core.ctx = &sink;
    at_node::FrameOutputs out;
    at_node::ImageBuffer image;
    if (time_n > 0) {  // the node's per-frame path, timed
      std::vector<double> ms, det_ms;
      for (int it = -count; it < time_n; ++it) {  // (the first pass over the frames is warm-up)
        const int f = ((it % count) + count) % count;
        const double stamp = 1000.0 + 0.02 * (it + count);
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = core.process(all.data() + (size_t)f * fb, fmt, stamp, stamp, &out,
                                    fmt == AT_FMT_BGR8 ? &image : nullptr);
        const auto t1 = std::chrono::steady_clock::now();
        if (rc != AT_OK && rc != AT_E_CAPACITY) {
          std::fprintf(stderr, "frame %d: %s\n", f, at_strerror(rc));
          return 1;
        }
        if (it >= 0) {
          ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
          det_ms.push_back(out.det_time_us * 1e-3);
        }
      }
      auto pct = [](std::vector<double> v, double q) {
        std::sort(v.begin(), v.end());
        return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
      };
      std::printf("{\"timing\":{\"calls\":%d,\"format\":\"%s\",\"width\":%d,\"height\":%d,\"p50_ms\":%.4f,"
                  "\"p99_ms\":%.4f,\"p50_detect_ms\":%.4f,\"detections_last\":%zu}}\n",
                  time_n, fmt_s.c_str(), W, H, pct(ms, 0.5), pct(ms, 0.99), pct(det_ms, 0.5), out.detections.size());
      return 0;
    }
    for (int f = 0; f < count; ++f) {
      const double stamp = 1000.0 + 0.02 * f;
      const int rc = core.process(all.data() + (size_t)f * fb, fmt, stamp, stamp, &out,
                                  fmt == AT_FMT_BGR8 ? &image : nullptr);
      if (rc != AT_OK && rc != AT_E_CAPACITY) {
        std::fprintf(stderr, "frame %d: %s\n", f, at_strerror(rc));
        return 1;
      }
      std::string dets = "[";
      char buf[512];
      for (size_t i = 0; i < out.detections.size(); ++i) {
        const at_detection& d = out.detections[i];
        std::snprintf(buf, sizeof(buf),
                      "%s{\"id\":%d,\"hamming\":%d,\"margin\":%.9g,\"c\":[%.17g,%.17g],\"p\":[[%.17g,%.17g],[%.17g,"
                      "%.17g],[%.17g,%.17g],[%.17g,%.17g]]}",
                      i ? "," : "", d.id, d.hamming, d.decision_margin, d.c[0], d.c[1], d.p[0][0], d.p[0][1],
                      d.p[1][0], d.p[1][1], d.p[2][0], d.p[2][1], d.p[3][0], d.p[3][1]);
        dets += buf;
      }
      dets += "]";
      std::string nt = "[";
      for (size_t i = 0; i < out.networktables_pose_data.size(); ++i) {
        std::snprintf(buf, sizeof(buf), "%s%.17g", i ? "," : "", out.networktables_pose_data[i]);
        nt += buf;
      }
      nt += "]";
      std::string hex;
      for (unsigned char c : out.proto) {
        std::snprintf(buf, sizeof(buf), "%02x", c);
        hex += buf;
      }
      std::printf("{\"frame\":%d,\"status\":%d,\"location\":\"%s\",\"pose_topic\":\"%s\",\"camera_pose_topic\":\"%s\","
                  "\"detections\":%s,\"robot\":%s,\"camera\":%s,\"networktables\":%s,\"proto_hex\":\"%s\"}\n",
                  f, rc, location.c_str(), core.pose_topic().c_str(), core.camera_pose_topic().c_str(), dets.c_str(),
                  sink.robot.c_str(), sink.camera.c_str(), nt.c_str(), hex.c_str());
      if (f == count - 1 && !proto_out.empty()) {
        std::ofstream po(proto_out, std::ios::binary);
        po.write(out.proto.data(), (std::streamsize)out.proto.size());
      }
      if (f == count - 1 && !image_out.empty() && !image.empty()) {
        std::ofstream io(image_out, std::ios::binary);
        io.write((const char*)image.data(), (std::streamsize)image.size());
      }
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
