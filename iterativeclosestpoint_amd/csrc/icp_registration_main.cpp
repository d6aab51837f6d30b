// icp_registration — the reference's standalone CLI (icp_registration.cpp:817-949) on the
// MI355X path: LAS in, stride down-sampling, ICP() with the CLI's rules on the GPU
// (icp_cli_icp), LAS + transformation report out. Same files, same order, same defaults;
// the reference's hard-coded names and parameters become flags with those defaults.
//
//   icp_registration [--source Scan_096_origin.las] [--target Scannew_099.las]
//                    [--sample-rate 50] [--max-iters 20] [--tolerance 1e-2]
//                    [--outdir .] [--device 0 | --devices 0,1,...] [--pause]
//
// --devices runs one registration over several GPUs of this process (icp_cli_icp_devices: the
// source sharded over them, the octree replicated, RCCL all-gathers per iteration).
//
// Exit code 255 (the reference's `return -1`) when an input cannot be read.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/icp_engine.h"
#include "../../include/icp_hip.h"
#include "../../include/icp_las.h"

namespace {

struct Args {
  std::string source = "Scan_096_origin.las";  // :825
  std::string target = "Scannew_099.las";      // :826
  long sample_rate = 50;                        // :858
  int max_iters = 20;                           // :900
  double tolerance = 1e-2;                      // :901
  std::string outdir = ".";
  std::vector<int> devices{0};
  bool pause = false;
};

[[noreturn]] void usage(const char* prog, int code) {
  std::fprintf(code ? stderr : stdout,
               "usage: %s [--source F] [--target F] [--sample-rate N] [--max-iters N] [--tolerance X]\n"
               "          [--outdir D] [--device N | --devices N,M,...] [--pause]\n",
               prog);
  std::exit(code);
}

Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; i++) {
    const std::string k = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) usage(argv[0], 2);
      return argv[++i];
    };
    if (k == "--source") a.source = val();
    else if (k == "--target") a.target = val();
    else if (k == "--sample-rate") a.sample_rate = std::strtol(val(), nullptr, 10);
    else if (k == "--max-iters") a.max_iters = (int)std::strtol(val(), nullptr, 10);
    else if (k == "--tolerance") a.tolerance = std::strtod(val(), nullptr);
    else if (k == "--outdir") a.outdir = val();
    else if (k == "--device") a.devices = {(int)std::strtol(val(), nullptr, 10)};
    else if (k == "--devices") {
      a.devices.clear();
      std::string list = val();
      size_t p = 0;
      while (p <= list.size()) {
        const size_t q = list.find(',', p);
        const std::string tok = list.substr(p, q == std::string::npos ? std::string::npos : q - p);
        char* end = nullptr;
        const long d = std::strtol(tok.c_str(), &end, 10);
        if (tok.empty() || *end != '\0' || d < 0) usage(argv[0], 2);
        a.devices.push_back((int)d);
        if (q == std::string::npos) break;
        p = q + 1;
      }
    }
    else if (k == "--pause") a.pause = true;
    else if (k == "-h" || k == "--help") usage(argv[0], 0);
    else usage(argv[0], 2);
  }
  if (a.sample_rate < 1) {
    std::fprintf(stderr, "--sample-rate must be >= 1\n");
    std::exit(2);
  }
  return a;
}

bool read_cloud(const std::string& path, std::vector<double>& xyz, icp_las_header& hdr) {
  std::cout << "  reading " << path << std::endl;
  if (icp_las_read_header(path.c_str(), ICP_LAS_CLI, &hdr) != 0) return false;
  xyz.resize((size_t)hdr.num_points * 3);
  const int64_t got = icp_las_read(path.c_str(), ICP_LAS_CLI, 0, xyz.data(), &hdr);
  if (got <= 0) return false;  // readLASFile returns read_count > 0 (:377)
  xyz.resize((size_t)got * 3);
  std::cout << "  " << got << " points, scale (" << hdr.scale[0] << ", " << hdr.scale[1] << ", " << hdr.scale[2]
            << "), offset (" << hdr.offset[0] << ", " << hdr.offset[1] << ", " << hdr.offset[2] << ")" << std::endl;
  return true;
}

int fail(const Args& a, const char* msg) {
  std::cout << "error: " << msg << std::endl;
  if (a.pause) std::cin.get();
  return -1;
}

std::string out_path(const Args& a, const char* name) { return a.outdir + "/" + name; }

}  // namespace

int main(int argc, char** argv) {
  const Args a = parse(argc, argv);
  std::cout << "=== ICP point-cloud fine registration (MI355X) ===" << std::endl;

  std::vector<double> src, tgt;
  icp_las_header hs{}, ht{};
  std::cout << "\nsource: " << a.source << std::endl;
  if (!read_cloud(a.source, src, hs)) return fail(a, "cannot read the source point cloud");
  std::cout << "\ntarget: " << a.target << std::endl;
  if (!read_cloud(a.target, tgt, ht)) return fail(a, "cannot read the target point cloud");

  // Stride down-sampling; both sampled clouds carry the SOURCE's scale/offset (:862-876).
  std::cout << "\ndown-sampling (1/" << a.sample_rate << ")..." << std::endl;
  std::vector<double> ss, ts;
  for (size_t i = 0; i < src.size() / 3; i += (size_t)a.sample_rate) ss.insert(ss.end(), &src[3 * i], &src[3 * i] + 3);
  for (size_t i = 0; i < tgt.size() / 3; i += (size_t)a.sample_rate) ts.insert(ts.end(), &tgt[3 * i], &tgt[3 * i] + 3);
  const int64_t ns = (int64_t)ss.size() / 3, nt = (int64_t)ts.size() / 3;
  std::cout << "source: " << ns << " points\ntarget: " << nt << " points" << std::endl;
  src.clear();
  src.shrink_to_fit();
  tgt.clear();
  tgt.shrink_to_fit();

  if (icp_las_write_cli(out_path(a, "sampled_source.las").c_str(), ss.data(), ns, hs.scale, hs.offset) != 0 ||
      icp_las_write_cli(out_path(a, "sampled_target.las").c_str(), ts.data(), nt, hs.scale, hs.offset) != 0)
    return fail(a, "cannot write the sampled clouds");

  std::cout << "\nparameters: max iterations=" << a.max_iters << ", tolerance=" << a.tolerance << std::endl;
  double R[9], t[3];
  const int cap = a.max_iters > 0 ? a.max_iters : 1;
  std::vector<double> transforms((size_t)cap * 16);
  int32_t n_tr = 0;
  if (a.devices.size() > 1) std::cout << "devices: " << a.devices.size() << " GPUs" << std::endl;
  const int rc = icp_cli_icp_devices(ss.data(), ns, ts.data(), nt, a.max_iters, a.tolerance, R, t, transforms.data(),
                                     cap, &n_tr, (int)a.devices.size(), a.devices.data());
  if (rc != 0) {
    std::cerr << "ICP failed (" << rc << "): " << icp_hip_last_error() << std::endl;
    return fail(a, "registration failed");
  }

  std::cout << "\n========== transform ==========" << std::endl << "R:" << std::endl;
  for (int i = 0; i < 3; i++)
    std::cout << "  [" << R[3 * i] << ", " << R[3 * i + 1] << ", " << R[3 * i + 2] << "]" << std::endl;
  std::cout << "\nt:\n  [" << t[0] << ", " << t[1] << ", " << t[2] << "]" << std::endl;
  std::cout << "===============================" << std::endl;

  // The source cloud was moved in place by ICP() (:598-605); the target is written unchanged.
  if (icp_las_write_cli(out_path(a, "registered_source.las").c_str(), ss.data(), ns, hs.scale, hs.offset) != 0 ||
      icp_las_write_cli(out_path(a, "registered_target.las").c_str(), ts.data(), nt, hs.scale, hs.offset) != 0 ||
      icp_write_transform_report(out_path(a, "icp_transformation.txt").c_str(), R, t, transforms.data(),
                                 n_tr < cap ? n_tr : cap) != 0)
    return fail(a, "cannot write the results");
  std::cout << "\ndone: registered_source.las, registered_target.las, icp_transformation.txt" << std::endl;
  if (a.pause) std::cin.get();
  return 0;
}
