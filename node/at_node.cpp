// at_node.cpp -- see at_node.h.  Host C++ only (the GPU work is behind at_api.h).
#include "at_node.h"

#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>

namespace at_node {

// ---------------------------------------------------------------------------
// minimal JSON reader (objects, arrays, strings, numbers, true/false/null): the
// two configuration files the node reads (the reference uses nlohmann::json)
// ---------------------------------------------------------------------------
namespace {
struct Json {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  double num = 0;
  bool is_int = false;  // numeric literal without fraction or exponent (nlohmann is_number_integer)
  bool b = false;
  std::string str;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;
  const Json* get(const std::string& k) const {
    if (kind != Obj) return nullptr;
    auto it = obj.find(k);
    return it == obj.end() ? nullptr : &it->second;
  }
};

struct Parser {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < e && *p == c) { ++p; return true; }
    return false;
  }
  std::string string_lit() {
    std::string s;
    if (!eat('"')) { ok = false; return s; }
    while (p < e && *p != '"') {
      if (*p == '\\' && p + 1 < e) {
        ++p;
        const char c = *p++;
        switch (c) {
          case 'n': s += '\n'; break;
          case 't': s += '\t'; break;
          case 'r': s += '\r'; break;
          case 'b': s += '\b'; break;
          case 'f': s += '\f'; break;
          case 'u': {  // keep ASCII, replace the rest
            unsigned v = 0;
            for (int k = 0; k < 4 && p < e; ++k, ++p) v = v * 16 + (unsigned)(isdigit(*p) ? *p - '0' : (tolower(*p) - 'a' + 10));
            s += v < 128 ? (char)v : '?';
            break;
          }
          default: s += c;
        }
      } else {
        s += *p++;
      }
    }
    if (p < e) ++p;
    else ok = false;
    return s;
  }
  Json value() {
    Json v;
    ws();
    if (p >= e) { ok = false; return v; }
    if (*p == '{') {
      ++p;
      v.kind = Json::Obj;
      if (eat('}')) return v;
      do {
        ws();
        std::string k = string_lit();
        if (!eat(':')) { ok = false; return v; }
        v.obj[k] = value();
      } while (ok && eat(','));
      if (!eat('}')) ok = false;
    } else if (*p == '[') {
      ++p;
      v.kind = Json::Arr;
      if (eat(']')) return v;
      do v.arr.push_back(value());
      while (ok && eat(','));
      if (!eat(']')) ok = false;
    } else if (*p == '"') {
      v.kind = Json::Str;
      v.str = string_lit();
    } else if (!strncmp(p, "true", 4)) {
      v.kind = Json::Bool; v.b = true; p += 4;
    } else if (!strncmp(p, "false", 5)) {
      v.kind = Json::Bool; p += 5;
    } else if (!strncmp(p, "null", 4)) {
      p += 4;
    } else {
      char* end = nullptr;
      v.num = strtod(p, &end);
      if (end == p) ok = false;
      v.kind = Json::Num;
      v.is_int = end != p && std::find_if(p, (const char*)end, [](char c) {
                               return c == '.' || c == 'e' || c == 'E';
                             }) == (const char*)end;
      p = end;
    }
    return v;
  }
};

bool parse_file(const std::string& path, Json* out, std::string* err) {
  std::ifstream f(path);
  if (!f) {
    if (err) *err = "cannot open " + path;
    return false;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  Parser ps{text.data(), text.data() + text.size()};
  *out = ps.value();
  if (!ps.ok) {
    if (err) *err = "malformed JSON in " + path;
    return false;
  }
  return true;
}

bool num_at(const Json* a, size_t i, double* v) {
  if (!a || a->kind != Json::Arr || i >= a->arr.size() || a->arr[i].kind != Json::Num) return false;
  *v = a->arr[i].num;
  return true;
}
}  // namespace

bool load_camera_calibration(const std::string& dir, const std::string& serial, at_camera* cam, std::string* err) {
  Json j;
  const std::string path = dir + "/calibrationmatrix_" + serial + ".json";
  if (!parse_file(path, &j, err)) return false;
  const Json* m = j.get("matrix");
  const Json* d = j.get("disto");
  if (!m || !d || m->kind != Json::Arr || m->arr.size() < 3 || d->kind != Json::Arr || d->arr.empty()) {
    if (err) *err = path + " needs 'matrix' and 'disto'";
    return false;
  }
  double fx, cx, fy, cy;  // apriltags_cuda_detector.cu:350-361: matrix[0][0], [0][2], [1][1], [1][2]
  const Json* d0 = &d->arr[0];
  if (!num_at(&m->arr[0], 0, &fx) || !num_at(&m->arr[0], 2, &cx) || !num_at(&m->arr[1], 1, &fy) ||
      !num_at(&m->arr[1], 2, &cy) || !num_at(d0, 0, &cam->k1) || !num_at(d0, 1, &cam->k2) ||
      !num_at(d0, 2, &cam->p1) || !num_at(d0, 3, &cam->p2) || !num_at(d0, 4, &cam->k3)) {
    if (err) *err = path + ": non-numeric calibration entries";
    return false;
  }
  cam->fx = fx; cam->cx = cx; cam->fy = fy; cam->cy = cy;
  return true;
}

bool load_extrinsics(const std::string& path, const std::string& serial, double R[9], double t[3],
                     std::string* location) {
  for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int i = 0; i < 3; ++i) t[i] = 0.0;
  if (location) location->clear();
  Json j;
  if (!parse_file(path, &j, nullptr)) return false;
  const Json* cmp = j.get("camera_mounted_positions");
  const Json* pos = cmp ? cmp->get(serial) : nullptr;
  std::string loc;
  if (pos && pos->kind == Json::Str) loc = pos->str;  // legacy format
  else if (pos && pos->get("location") && pos->get("location")->kind == Json::Str) loc = pos->get("location")->str;
  else return false;
  if (location) *location = loc;
  const Json* ex = j.get("extrinsics");
  const Json* e = ex ? ex->get(loc) : nullptr;
  const Json* rot = e ? e->get("rotation") : nullptr;
  const Json* off = e ? e->get("offset") : nullptr;
  if (!rot || !off) return false;
  double Rt[9], tt[3];
  // rotation: 3x3 nested or flat 9
  if (rot->kind == Json::Arr && rot->arr.size() == 3) {
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        if (!num_at(&rot->arr[r], c, &Rt[3 * r + c])) return false;
  } else {
    for (int k = 0; k < 9; ++k)
      if (!num_at(rot, k, &Rt[k])) return false;
  }
  for (int k = 0; k < 3; ++k)
    if (!num_at(off, k, &tt[k])) return false;
  std::copy(Rt, Rt + 9, R);
  std::copy(tt, tt + 3, t);
  return true;
}

std::string package_share_directory(const std::string& package) {
  const char* env = std::getenv("AMENT_PREFIX_PATH");
  if (!env) return "";
  std::stringstream ss(env);
  std::string prefix;
  while (std::getline(ss, prefix, ':')) {
    if (prefix.empty()) continue;
    const std::string marker = prefix + "/share/ament_index/resource_index/packages/" + package;
    if (access(marker.c_str(), F_OK) == 0) return prefix + "/share/" + package;
  }
  return "";
}

bool load_camera_config(const std::string& path, const std::string& serial, CameraConfig* out) {
  Json j;
  if (!parse_file(path, &j, nullptr)) return false;
  const Json* cmp = j.get("camera_mounted_positions");
  const Json* c = cmp ? cmp->get(serial) : nullptr;
  if (!c || c->kind != Json::Obj) return false;
  auto str = [&](const char* k, std::string* v) {
    const Json* e = c->get(k);
    if (!e || e->kind != Json::Str) return false;
    *v = e->str;
    return true;
  };
  auto integer = [&](const char* k, int* v) {
    const Json* e = c->get(k);
    if (!e || e->kind != Json::Num || !e->is_int) return false;
    *v = (int)e->num;
    return true;
  };
  CameraConfig cfg;
  if (!str("location", &cfg.location) || !str("format", &cfg.format) || !integer("height", &cfg.height) ||
      !integer("width", &cfg.width) || !integer("frame_rate", &cfg.frame_rate) ||
      !str("api_preference", &cfg.api_preference))
    return false;  // incomplete records are skipped (config_loader.cpp:83-94)
  *out = cfg;
  return true;
}

NetworkTablesConfig load_network_tables_config(const std::string& path) {
  NetworkTablesConfig nt;
  Json j;
  if (!parse_file(path, &j, nullptr)) return nt;
  const Json* c = j.get("network_tables_config");
  if (const Json* a = c ? c->get("table_address") : nullptr)
    if (a->kind == Json::Str) nt.table_address = a->str;
  if (const Json* n = c ? c->get("table_name") : nullptr)
    if (n->kind == Json::Str) nt.table_name = n->str;
  return nt;
}

bool resolve_node_config(const std::string& serial, const std::string& share_dir, NodeConfig* out, std::string* err) {
  NodeConfig& nc = *out;
  nc = NodeConfig{};
  nc.share_dir = share_dir.empty() ? package_share_directory("vision_config_data") : share_dir;
  if (nc.share_dir.empty()) {
    if (err) *err = "package vision_config_data not found (AMENT_PREFIX_PATH) and no config directory given";
    return false;
  }
  nc.system_config = nc.share_dir + "/data/system_config.json";
  nc.calibration_dir = nc.share_dir + "/data/calibration";
  if (!load_camera_calibration(nc.calibration_dir, serial, &nc.cam, err)) return false;
  nc.have_extrinsics = load_extrinsics(nc.system_config, serial, nc.R, nc.t, &nc.location);
  nc.networktables = load_network_tables_config(nc.system_config);
  if (!load_camera_config(nc.system_config, serial, &nc.camera)) {  // apriltags_cuda_detector.cu:159-169
    if (err) *err = "Failed to load camera configuration for serial: " + serial;
    return false;
  }
  return true;
}

bool apply_cpu_pinning_and_scheduling(int pin_to_core, int priority, std::string* log) {
  auto say = [&](const std::string& m) {
    if (log) *log += m + "\n";
  };
  if (pin_to_core == -1) {
    say("CPU pinning disabled (pin_to_core = -1)");
    return true;
  }
  bool ok = true;
  const int ncores = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (pin_to_core < 0 || pin_to_core >= ncores) {
    say("Invalid CPU core " + std::to_string(pin_to_core) + ". System has " + std::to_string(ncores) + " cores");
    ok = false;
  } else {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(pin_to_core, &set);
    const int r = pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    if (r) {
      say(std::string("Failed to set CPU affinity: ") + std::strerror(r));
      ok = false;
    } else {
      say("Pinned to CPU core " + std::to_string(pin_to_core));
    }
  }
  const int lo = sched_get_priority_min(SCHED_FIFO), hi = sched_get_priority_max(SCHED_FIFO);
  if (priority < lo || priority > hi) {
    say("Invalid priority " + std::to_string(priority) + " for SCHED_FIFO");
    ok = false;
  } else {
    sched_param sp{};
    sp.sched_priority = priority;
    const int r = pthread_setschedparam(pthread_self(), SCHED_FIFO, &sp);
    if (r) {
      say(std::string("Failed to set real-time scheduling: ") + std::strerror(r) +
          " (needs root or CAP_SYS_NICE)");
      ok = false;
    } else {
      say("SCHED_FIFO priority " + std::to_string(priority));
    }
  }
  if (ok) {  // verifySettings (:124-171)
    cpu_set_t set;
    CPU_ZERO(&set);
    int policy = 0;
    sched_param sp{};
    if (pthread_getaffinity_np(pthread_self(), sizeof(set), &set) || !CPU_ISSET(pin_to_core, &set) ||
        pthread_getschedparam(pthread_self(), &policy, &sp) || policy != SCHED_FIFO || sp.sched_priority != priority) {
      say("verification of affinity / scheduling failed");
      ok = false;
    }
  }
  return ok;
}

// ---------------------------------------------------------------------------
// ApriltagListProto wire format (proto2)
// ---------------------------------------------------------------------------
namespace {
void put_varint(std::string* s, uint64_t v) {
  while (v >= 0x80) {
    s->push_back((char)(uint8_t)(v | 0x80));
    v >>= 7;
  }
  s->push_back((char)(uint8_t)v);
}
void put_double(std::string* s, int field, double v) {
  put_varint(s, ((uint64_t)field << 3) | 1);  // wire type 1: 64-bit
  uint64_t u;
  std::memcpy(&u, &v, 8);
  for (int i = 0; i < 8; ++i) s->push_back((char)(uint8_t)(u >> (8 * i)));
}
}  // namespace

std::string encode_apriltag_list(const at_tag_detection* tags, int n, double collect_time) {
  std::string out;
  for (int i = 0; i < n; ++i) {
    std::string m;
    put_double(&m, 1, collect_time);
    put_varint(&m, (2u << 3) | 0);                       // tag_id, varint
    put_varint(&m, (uint64_t)(int64_t)tags[i].id);       // int32: negative -> 10-byte sign extension
    put_double(&m, 3, tags[i].robot[0]);
    put_double(&m, 4, tags[i].robot[1]);
    put_double(&m, 5, tags[i].robot[2]);
    put_varint(&out, (1u << 3) | 2);                     // tags, length-delimited
    put_varint(&out, m.size());
    out += m;
  }
  return out;
}

// ---------------------------------------------------------------------------
// outlines
// ---------------------------------------------------------------------------
namespace {
void plot(uint8_t* bgr, int W, int H, int x, int y, const uint8_t c[3]) {
  if (x < 0 || y < 0 || x >= W || y >= H) return;
  uint8_t* p = bgr + ((size_t)y * W + x) * 3;
  p[0] = c[0]; p[1] = c[1]; p[2] = c[2];
}
// segment of the given thickness: every pixel centre within thickness/2 of the segment
void thick_line(uint8_t* bgr, int W, int H, double x0, double y0, double x1, double y1, double thick,
                const uint8_t c[3]) {
  const double r = thick / 2.0;
  const int xa = (int)std::floor(std::min(x0, x1) - r), xb = (int)std::ceil(std::max(x0, x1) + r);
  const int ya = (int)std::floor(std::min(y0, y1) - r), yb = (int)std::ceil(std::max(y0, y1) + r);
  const double dx = x1 - x0, dy = y1 - y0, l2 = dx * dx + dy * dy;
  for (int y = std::max(ya, 0); y <= std::min(yb, H - 1); ++y)
    for (int x = std::max(xa, 0); x <= std::min(xb, W - 1); ++x) {
      double u = l2 > 0 ? ((x - x0) * dx + (y - y0) * dy) / l2 : 0.0;
      u = std::min(1.0, std::max(0.0, u));
      const double ex = x0 + u * dx - x, ey = y0 + u * dy - y;
      if (ex * ex + ey * ey <= r * r) plot(bgr, W, H, x, y, c);
    }
}
// digit strokes on a 0..4 x 0..8 grid (single-stroke "simplex" digits)
const std::vector<std::vector<std::pair<int, int>>>& digit_strokes(int d) {
  static const std::vector<std::vector<std::vector<std::pair<int, int>>>> k = {
      {{{0, 1}, {1, 0}, {3, 0}, {4, 1}, {4, 7}, {3, 8}, {1, 8}, {0, 7}, {0, 1}}},             // 0
      {{{1, 2}, {2, 0}, {2, 8}}, {{1, 8}, {3, 8}}},                                       // 1
      {{{0, 1}, {1, 0}, {3, 0}, {4, 1}, {4, 3}, {0, 8}, {4, 8}}},                         // 2
      {{{0, 0}, {4, 0}, {2, 3}, {3, 3}, {4, 4}, {4, 7}, {3, 8}, {1, 8}, {0, 7}}},         // 3
      {{{3, 8}, {3, 0}, {0, 5}, {4, 5}}},                                                 // 4
      {{{4, 0}, {0, 0}, {0, 3}, {3, 3}, {4, 4}, {4, 7}, {3, 8}, {0, 8}}},                 // 5
      {{{4, 0}, {2, 0}, {0, 3}, {0, 7}, {1, 8}, {3, 8}, {4, 7}, {4, 5}, {3, 4}, {0, 4}}}, // 6
      {{{0, 0}, {4, 0}, {1, 8}}},                                                         // 7
      {{{1, 4}, {0, 3}, {0, 1}, {1, 0}, {3, 0}, {4, 1}, {4, 3}, {3, 4}, {1, 4}, {0, 5}, {0, 7}, {1, 8},
        {3, 8}, {4, 7}, {4, 5}, {3, 4}}},                                                  // 8
      {{{4, 4}, {1, 4}, {0, 3}, {0, 1}, {1, 0}, {3, 0}, {4, 1}, {4, 5}, {2, 8}, {0, 8}}}, // 9
  };
  return k[d];
}
}  // namespace

void draw_detection_outlines(uint8_t* bgr, int W, int H, const at_detection* dets, int n) {
  static const uint8_t kGreen[3] = {0, 0xff, 0}, kRed[3] = {0, 0, 0xff}, kBlue[3] = {0xff, 0, 0},
                       kText[3] = {0xff, 0x99, 0};
  for (int i = 0; i < n; ++i) {
    const at_detection& d = dets[i];
    // cv::Point(double, double) truncates to int (apriltag_utils.cu:58-65)
    auto P = [&](int k, int c) { return (double)(int)d.p[k][c]; };
    thick_line(bgr, W, H, P(0, 0), P(0, 1), P(1, 0), P(1, 1), 2, kGreen);
    thick_line(bgr, W, H, P(0, 0), P(0, 1), P(3, 0), P(3, 1), 2, kRed);
    thick_line(bgr, W, H, P(1, 0), P(1, 1), P(2, 0), P(2, 1), 2, kBlue);
    thick_line(bgr, W, H, P(2, 0), P(2, 1), P(3, 0), P(3, 1), 2, kBlue);
    // id text centred on c (:67-77), about the height of FONT_HERSHEY_* at scale 1
    const std::string text = std::to_string(d.id);
    const double sc = 2.5, adv = 7 * sc;
    const double tw = adv * text.size() - 2 * sc, th = 8 * sc;
    const double ox = (int)(d.c[0] - tw / 2), oy = (int)(d.c[1] - th / 2);
    for (size_t k = 0; k < text.size(); ++k) {
      if (text[k] < '0' || text[k] > '9') continue;  // '-' never occurs: ids are >= 0
      for (const auto& stroke : digit_strokes(text[k] - '0'))
        for (size_t s = 1; s < stroke.size(); ++s)
          thick_line(bgr, W, H, ox + k * adv + stroke[s - 1].first * sc, oy + stroke[s - 1].second * sc,
                     ox + k * adv + stroke[s].first * sc, oy + stroke[s].second * sc, 2, kText);
    }
  }
}

// ---------------------------------------------------------------------------
// DetectorCore
// ---------------------------------------------------------------------------
DetectorCore::DetectorCore(int width, int height, const Params& params, const at_camera& cam,
                           const double extr_R[9], const double extr_t[3], int device)
    : width_(width), height_(height), params_(params) {
  for (int i = 0; i < 9; ++i) R_[i] = extr_R ? extr_R[i] : ((i % 4 == 0) ? 1.0 : 0.0);
  for (int i = 0; i < 3; ++i) t_[i] = extr_t ? extr_t[i] : 0.0;
  init(cam, device);
}

DetectorCore::DetectorCore(const Params& params, const NodeConfig& config, int device)
    : width_(config.camera.width), height_(config.camera.height), params_(params) {
  std::copy(config.R, config.R + 9, R_);
  std::copy(config.t, config.t + 3, t_);
  init(config.cam, device);
}

void DetectorCore::init(const at_camera& cam, int device) {
  at_config cfg;
  at_config_default(&cfg, width_, height_);  // the node's detector settings (:139-147), TAGSIZE
  cfg.device = device;
  const int rc = at_create(&cfg, &cam, &det_);
  if (rc != AT_OK) throw std::runtime_error(std::string("at_create: ") + at_strerror(rc));
  dets_.resize(at_max_detections());  // every detection of a frame (no truncation)
  poses_.resize(at_max_detections());
  if (params_.measurement_mode) {
    csv_path_ = params_.timing_csv_path;
    if (csv_path_.empty()) {  // apriltags_timing_YYYYMMDD_hhmmss.csv (:565-574)
      const std::time_t now = std::time(nullptr);
      std::tm tm_now;
      localtime_r(&now, &tm_now);
      char buf[64];
      std::strftime(buf, sizeof(buf), "apriltags_timing_%Y%m%d_%H%M%S.csv", &tm_now);
      csv_path_ = buf;
    }
    csv_ = std::fopen(csv_path_.c_str(), "w");
    if (csv_) {
      std::fputs("latency_us,det_time_us,publish_pose_us,publish_camera_pose_us,publish_image_us,"
                 "networktables_us,processing_time_us\n", csv_);
      std::fflush(csv_);
    }
  }
}

DetectorCore::~DetectorCore() {
  image_queue_.reset();  // stops the publisher thread (the reference stops its queue, :80-82)
  if (csv_) std::fclose(csv_);
  at_destroy(det_);
}

int DetectorCore::process(const uint8_t* frame, at_pixfmt fmt, double stamp_s, double receive_s, FrameOutputs* out,
                          ImageBuffer* annotate) {
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b) {
    return (long long)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
  };
  const auto start = clk::now();
  *out = FrameOutputs{};
  int n = 0;
  const auto det0 = clk::now();
  int rc = at_detect(det_, frame, fmt, dets_.data(), (int)dets_.size(), &n);
  const auto det1 = clk::now();
  out->status = rc;
  out->det_time_us = us(det0, det1);
  if (rc != AT_OK && rc != AT_E_CAPACITY) return rc;
  n = std::min(n, (int)dets_.size());
  out->detections.assign(dets_.begin(), dets_.begin() + n);
  const int np = at_poses(det_, 0, poses_.data(), n);
  if (np < 0) return np;
  out->tags.resize(np);
  if (np > 0) at_tag_detections(poses_.data(), np, R_, t_, out->tags.data());  // closest first
  for (const at_tag_detection& d : out->tags) {
    out->networktables_pose_data.insert(out->networktables_pose_data.end(),
                                        {stamp_s, d.id * 1.0, d.robot[0], d.robot[1], d.robot[2]});
    out->camera.push_back({d.id, d.camera[0], d.camera[1], d.camera[2]});
    out->robot.push_back({d.id, d.robot[0], d.robot[1], d.robot[2]});
  }
  out->proto = encode_apriltag_list(out->tags.data(), (int)out->tags.size(), stamp_s);
  if (annotate && fmt == AT_FMT_BGR8) {
    // draw_detection_outlines (:411) on the GPU, on the copy of the frame at_detect
    // staged in HBM: no host copy of the frame, no host drawing
    annotate->resize((size_t)width_ * height_ * 3);
    const int arc = at_annotate_staged(det_, 0, out->detections.data(), n, annotate->data());
    if (arc != AT_OK) return arc;
  }
  const auto nt0 = clk::now();
  if (send_networktables) send_networktables(ctx, out->networktables_pose_data, out->proto);
  const auto nt1 = clk::now();
  if (publish_robot) publish_robot(ctx, out->robot);
  const auto pp1 = clk::now();
  if (publish_camera) publish_camera(ctx, out->camera);
  const auto pc1 = clk::now();
  if (publish_image && annotate && !annotate->empty()) {
    if (!image_queue_) {
      auto pub = publish_image;
      void* c = ctx;
      image_queue_.reset(new PublisherQueue<StampedImage>(
          [pub, c](const StampedImage& img) { pub(c, img.bgr, img.stamp_s); }, 2));
    }
    // image_pub_queue_->enqueue (:514-518): the queue owns a copy
    image_queue_->enqueue(StampedImage{std::vector<uint8_t>(annotate->begin(), annotate->end()), stamp_s});
  }
  const auto pi1 = clk::now();
  if (csv_) {  // latency,det,publish_pose,publish_camera_pose,publish_image,networktables,processing (:526-552)
    std::fprintf(csv_, "%lld,%lld,%lld,%lld,%lld,%lld,%lld\n", (long long)std::llround((receive_s - stamp_s) * 1e6),
                 us(det0, det1), us(nt1, pp1), us(pp1, pc1), us(pc1, pi1), us(nt0, nt1), us(start, pi1));
    std::fflush(csv_);
  }
  return rc;
}

}  // namespace at_node

// ---------------------------------------------------------------------------
// C entry points of libat_node.so (tests and non-C++ callers)
// ---------------------------------------------------------------------------
extern "C" {

long long at_node_encode_apriltag_list(const at_tag_detection* tags, int n, double collect_time, uint8_t* out,
                                       size_t cap) {
  const std::string s = at_node::encode_apriltag_list(tags, n, collect_time);
  if (out && cap >= s.size()) std::memcpy(out, s.data(), s.size());
  return (long long)s.size();
}

int at_node_load_camera_calibration(const char* dir, const char* serial, at_camera* cam) {
  return at_node::load_camera_calibration(dir, serial, cam, nullptr) ? 0 : -1;
}

int at_node_load_extrinsics(const char* path, const char* serial, double* R, double* t, char* location,
                            size_t cap) {
  std::string loc;
  const bool ok = at_node::load_extrinsics(path, serial, R, t, &loc);
  if (location && cap) {
    std::strncpy(location, loc.c_str(), cap - 1);
    location[cap - 1] = 0;
  }
  return ok ? 0 : -1;
}

void at_node_draw_detection_outlines(uint8_t* bgr, int width, int height, const at_detection* dets, int n) {
  at_node::draw_detection_outlines(bgr, width, height, dets, n);
}

// ConfigLoader::getCameraConfig: width, height, frame_rate and the location string.
int at_node_load_camera_config(const char* path, const char* serial, int* width, int* height, int* frame_rate,
                               char* location, size_t cap) {
  at_node::CameraConfig c;
  if (!at_node::load_camera_config(path, serial, &c)) return -1;
  if (width) *width = c.width;
  if (height) *height = c.height;
  if (frame_rate) *frame_rate = c.frame_rate;
  if (location && cap) {
    std::strncpy(location, c.location.c_str(), cap - 1);
    location[cap - 1] = 0;
  }
  return 0;
}

// package_share_directory("vision_config_data") through $AMENT_PREFIX_PATH.
long long at_node_package_share_directory(const char* package, char* out, size_t cap) {
  const std::string s = at_node::package_share_directory(package);
  if (out && cap) {
    std::strncpy(out, s.c_str(), cap - 1);
    out[cap - 1] = 0;
  }
  return (long long)s.size();
}

// resolve_node_config: W x H, intrinsics (fx fy cx cy k1 k2 p1 p2 k3), extrinsics.
int at_node_resolve_config(const char* serial, const char* share_dir, int* wh, at_camera* cam, double* R, double* t,
                           int* have_extrinsics) {
  at_node::NodeConfig nc;
  if (!at_node::resolve_node_config(serial, share_dir ? share_dir : "", &nc, nullptr)) return -1;
  if (wh) {
    wh[0] = nc.camera.width;
    wh[1] = nc.camera.height;
  }
  if (cam) *cam = nc.cam;
  if (R) std::copy(nc.R, nc.R + 9, R);
  if (t) std::copy(nc.t, nc.t + 3, t);
  if (have_extrinsics) *have_extrinsics = nc.have_extrinsics;
  return 0;
}

// apply_cpu_pinning_and_scheduling on the calling thread; 1 = applied and verified.
int at_node_apply_cpu_pinning(int pin_to_core, int priority, char* log, size_t cap) {
  std::string msg;
  const bool ok = at_node::apply_cpu_pinning_and_scheduling(pin_to_core, priority, &msg);
  if (log && cap) {
    std::strncpy(log, msg.c_str(), cap - 1);
    log[cap - 1] = 0;
  }
  return ok ? 1 : 0;
}

}  // extern "C"
