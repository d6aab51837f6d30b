// lasio.cpp — LAS 1.2 I/O and the transformation report of the reference front-ends
// (include/icp_las.h). Host code; byte layout and arithmetic follow the reference exactly.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <vector>

#include "../../include/icp_las.h"

namespace {

template <typename T>
T rd(const char* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

template <typename T>
void wr(char* p, T v) {
  std::memcpy(p, &v, sizeof(T));
}

int parse_header(const char* h, int rules, icp_las_header* out) {
  if (rules == ICP_LAS_CORE && std::strncmp(h, "LASF", 4) != 0) return -2;  // lasio.cpp:31-35
  out->offset_to_points = rd<uint32_t>(h + 96);
  out->num_points = rd<uint32_t>(h + 107);
  out->record_length = rd<uint16_t>(h + 105);
  for (int a = 0; a < 3; a++) {
    out->scale[a] = rd<double>(h + 131 + 8 * a);
    out->offset[a] = rd<double>(h + 155 + 8 * a);
    out->max[a] = rd<double>(h + 179 + 16 * a);
    out->min[a] = rd<double>(h + 187 + 16 * a);
  }
  if (rules == ICP_LAS_CLI && (out->num_points == 0 || out->num_points > 100000000u)) return -2;  // :291
  return 0;
}

}  // namespace

extern "C" {

int icp_las_read_header(const char* path, int rules, icp_las_header* hdr) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) return -1;
  char h[227];
  f.read(h, 227);
  if (!f) return -1;
  return parse_header(h, rules, hdr);
}

int64_t icp_las_read(const char* path, int rules, int64_t max_points, double* xyz, icp_las_header* hdr) {
  icp_las_header local;
  icp_las_header* H = hdr ? hdr : &local;
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) return -1;
  char h[227];
  f.read(h, 227);
  if (!f) return -1;
  const int rc = parse_header(h, rules, H);
  if (rc != 0) return rc;
  f.seekg(H->offset_to_points, std::ios::beg);
  if (!f) return -1;
  int64_t n = H->num_points;
  // lasio.cpp:60-63 (core rules). The CLI reader has no limit (icp_registration.cpp:286-366), but
  // max_points is also the caller's buffer capacity (icp_las.h): never read past it (found by the
  // ASan build, tests/test_sanitize.py)
  if (max_points > 0 && max_points < n) n = max_points;
  // Batches of 10000 records (lasio.cpp:70-103 / :326-366). A short read at end of file still
  // parses the whole batch from the (zero-initialised, then reused) buffer, as the reference.
  const int kBatch = 10000;
  const int rl = H->record_length;
  std::vector<char> buf((size_t)kBatch * (size_t)(rl > 0 ? rl : 1), 0);
  int64_t got = 0;
  for (int64_t b = 0; b < n; b += kBatch) {
    const int cnt = (int)((n - b) < kBatch ? (n - b) : kBatch);
    f.read(buf.data(), (std::streamsize)cnt * rl);
    if (!f && !f.eof()) break;
    for (int i = 0; i < cnt; i++) {
      const char* r = buf.data() + (size_t)i * rl;
      const int32_t X = rl >= 12 ? rd<int32_t>(r) : 0;
      const int32_t Y = rl >= 12 ? rd<int32_t>(r + 4) : 0;
      const int32_t Z = rl >= 12 ? rd<int32_t>(r + 8) : 0;
      double* p = xyz + 3 * got;
      p[0] = X * H->scale[0] + H->offset[0];
      p[1] = Y * H->scale[1] + H->offset[1];
      p[2] = Z * H->scale[2] + H->offset[2];
      got++;
    }
  }
  return got;
}

int icp_las_write_core_bounds(const char* path, const double* xyz, int64_t n, const double bounds[6]) {
  if (n <= 0) return -2;  // lasio.cpp:129-132
  if (!bounds) return -1;
  const double mn[3] = {bounds[0], bounds[2], bounds[4]}, mx[3] = {bounds[1], bounds[3], bounds[5]};
  std::ofstream f(path, std::ios::binary);
  if (!f.is_open()) return -1;
  char h[227];
  std::memset(h, 0, sizeof(h));
  std::memcpy(h, "LASF", 4);
  h[24] = 1;
  h[25] = 2;
  wr<uint16_t>(h + 94, 227);
  wr<uint32_t>(h + 96, 227);
  h[104] = 0;
  wr<uint16_t>(h + 105, 20);
  wr<uint32_t>(h + 107, (uint32_t)n);
  for (int a = 0; a < 3; a++) {
    wr<double>(h + 131 + 8 * a, 0.001);
    wr<double>(h + 155 + 8 * a, mn[a]);
    wr<double>(h + 179 + 16 * a, mx[a]);
    wr<double>(h + 187 + 16 * a, mn[a]);
  }
  f.write(h, 227);
  std::vector<char> rec((size_t)n * 20, 0);
  for (int64_t i = 0; i < n; i++)
    for (int a = 0; a < 3; a++)
      wr<int32_t>(rec.data() + 20 * i + 4 * a, (int32_t)((xyz[3 * i + a] - mn[a]) / 0.001));
  f.write(rec.data(), (std::streamsize)rec.size());
  return f ? 0 : -1;
}

int icp_las_write_core(const char* path, const double* xyz, int64_t n) {
  if (n <= 0) return -2;  // lasio.cpp:129-132
  // PointCloud::computeBounds (pointcloud.cpp:24-45): std::min / std::max
  double b[6];
  for (int a = 0; a < 3; a++) {
    b[2 * a] = std::numeric_limits<double>::max();
    b[2 * a + 1] = std::numeric_limits<double>::lowest();
  }
  for (int64_t i = 0; i < n; i++)
    for (int a = 0; a < 3; a++) {
      const double v = xyz[3 * i + a];
      b[2 * a] = (v < b[2 * a]) ? v : b[2 * a];
      b[2 * a + 1] = (b[2 * a + 1] < v) ? v : b[2 * a + 1];
    }
  return icp_las_write_core_bounds(path, xyz, n, b);
}

int icp_las_write_cli(const char* path, const double* xyz, int64_t n, const double scale[3], const double offset[3]) {
  if (n <= 0) return -2;  // the reference reads points[0] unconditionally (:762)
  std::ofstream f(path, std::ios::binary);
  if (!f.is_open()) return -1;
  char h[227];
  std::memset(h, 0, sizeof(h));
  std::memcpy(h, "LASF", 4);
  h[24] = 1;
  h[25] = 2;
  const char* sys = "ICP Registration";
  std::memcpy(h + 26, sys, std::strlen(sys));
  const char* sw = "Custom ICP";
  std::memcpy(h + 58, sw, std::strlen(sw));
  wr<uint16_t>(h + 90, 307);
  wr<uint16_t>(h + 92, 2025);
  wr<uint16_t>(h + 94, 227);
  wr<uint32_t>(h + 96, 227);
  wr<uint32_t>(h + 100, 0);
  h[104] = 0;
  wr<uint16_t>(h + 105, 20);
  wr<uint32_t>(h + 107, (uint32_t)n);
  double mn[3], mx[3];
  for (int a = 0; a < 3; a++) mn[a] = mx[a] = xyz[a];
  for (int64_t i = 0; i < n; i++)
    for (int a = 0; a < 3; a++) {
      const double v = xyz[3 * i + a];
      if (v < mn[a]) mn[a] = v;
      if (v > mx[a]) mx[a] = v;
    }
  for (int a = 0; a < 3; a++) {
    wr<double>(h + 131 + 8 * a, scale[a]);
    wr<double>(h + 155 + 8 * a, offset[a]);
    wr<double>(h + 179 + 16 * a, mx[a]);
    wr<double>(h + 187 + 16 * a, mn[a]);
  }
  f.write(h, 227);
  std::vector<char> rec((size_t)n * 20, 0);
  for (int64_t i = 0; i < n; i++)
    for (int a = 0; a < 3; a++)
      wr<int32_t>(rec.data() + 20 * i + 4 * a, (int32_t)((xyz[3 * i + a] - offset[a]) / scale[a]));
  f.write(rec.data(), (std::streamsize)rec.size());
  return f ? 0 : -1;
}

int icp_write_transform_report(const char* path, const double R[9], const double t[3], const double* T,
                               int32_t n_T) {
  // saveTransformation (icp_registration.cpp:625-695): same labels, same stream formatting
  std::ofstream file(path);
  if (!file.is_open()) return -1;
  file << "ICP配准变换参数" << std::endl;
  file << "==================" << std::endl << std::endl;
  file << "说明: 将源点云变换到目标点云坐标系下的变换矩阵" << std::endl;
  file << "变换公式: P_target = R * P_source + t" << std::endl << std::endl;
  if (T != nullptr && n_T > 0) {
    file << "==================" << std::endl;
    file << "迭代过程变换参数" << std::endl;
    file << "==================" << std::endl << std::endl;
    file.precision(10);
    for (int32_t it = 0; it < n_T; it++) {
      const double* M = T + 16 * it;
      file << "--- 迭代 " << (it + 1) << " ---" << std::endl;
      file << "旋转矩阵 R:" << std::endl;
      for (int i = 0; i < 3; i++) {
        file << "  [";
        for (int j = 0; j < 3; j++) {
          file << M[4 * i + j];
          if (j < 2) file << ", ";
        }
        file << "]" << std::endl;
      }
      file << "平移向量 t:" << std::endl;
      file << "  [" << M[3] << ", " << M[7] << ", " << M[11] << "]" << std::endl;
      file << std::endl;
    }
    file << std::endl;
  }
  file << "==================" << std::endl;
  file << "最终变换参数" << std::endl;
  file << "==================" << std::endl << std::endl;
  file << "旋转矩阵 R (3x3):" << std::endl;
  file.precision(10);
  for (int i = 0; i < 3; i++) {
    file << "  [";
    for (int j = 0; j < 3; j++) {
      file << R[3 * i + j];
      if (j < 2) file << ", ";
    }
    file << "]" << std::endl;
  }
  file << std::endl << "平移向量 t (3x1):" << std::endl;
  file << "  [" << t[0] << ", " << t[1] << ", " << t[2] << "]" << std::endl;
  file << std::endl << "变换矩阵 (齐次坐标形式 4x4):" << std::endl;
  for (int i = 0; i < 3; i++) {
    file << "  [";
    for (int j = 0; j < 3; j++) file << R[3 * i + j] << ", ";
    file << t[i] << "]" << std::endl;
  }
  file << "  [0, 0, 0, 1]" << std::endl;
  return file ? 0 : -1;
}

}  // extern "C"
