// shard_driver.cpp — one rank of the multi-GPU scan-to-map as a C++ program: what a MapOptimization
// node running one process per GPU does with include/llsr_rccl.h. Test
// infrastructure: tests/test_gpu_rccl.py runs it at world 1 on the GPU box and compares the reports
// with the oracle's statement of the split mode.
//
//   llsr_shard_driver IN OUT MODE ITERS POLL [WORLD RANK ID_FILE]
//
// IN: int32 P, then per problem int32 n[4] (corner queries, surf queries, corner map, surf map),
// the four float4 clouds, float pose[6]. OUT: P llsr_lm_report records, then float allreduce_us.
// WORLD > 1: rank 0 writes the ncclUniqueId to ID_FILE, the other ranks wait for it; rank r uses
// HIP device r.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "llsr.h"
#include "llsr_rccl.h"

#define CHECK(cond, msg)                                     \
  do {                                                       \
    if (!(cond)) {                                           \
      std::fprintf(stderr, "shard_driver: %s\n", msg);       \
      return 1;                                              \
    }                                                        \
  } while (0)

struct Problem {
  std::vector<float> cloud[4];
  float pose[6];
};

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s IN OUT MODE ITERS POLL [WORLD RANK ID_FILE]\n", argv[0]);
    return 2;
  }
  const int mode = std::atoi(argv[3]), iters = std::atoi(argv[4]), poll = std::atoi(argv[5]);
  const int world = argc > 6 ? std::atoi(argv[6]) : 1, rank = argc > 7 ? std::atoi(argv[7]) : 0;
  const std::string id_file = argc > 8 ? argv[8] : "";
  std::ifstream in(argv[1], std::ios::binary);
  CHECK(in.good(), "cannot open IN");
  int32_t P = 0;
  in.read(reinterpret_cast<char*>(&P), 4);
  CHECK(P > 0 && P < 100000, "bad problem count");
  std::vector<Problem> probs(P);
  for (auto& pr : probs) {
    int32_t n[4];
    in.read(reinterpret_cast<char*>(n), sizeof n);
    for (int k = 0; k < 4; ++k) {
      CHECK(n[k] >= 0, "bad cloud size");
      pr.cloud[k].resize(4 * (size_t)n[k]);
      in.read(reinterpret_cast<char*>(pr.cloud[k].data()), pr.cloud[k].size() * sizeof(float));
    }
    in.read(reinterpret_cast<char*>(pr.pose), sizeof pr.pose);
  }
  CHECK(in.good(), "short IN");

  CHECK(hipSetDevice(rank) == hipSuccess, "hipSetDevice");
  llsr_config cfg;
  llsr_config_default(&cfg, LLSR_LIDAR_VLP16);
  cfg.mode = mode;
  cfg.iterCountThres = iters;
  llsr_handle* h = nullptr;
  CHECK(llsr_create(&cfg, rank, 1, 1, &h) == LLSR_OK, "llsr_create");

  // pack the four kinds of clouds with int64 offsets [P+1], as llsr_s2m_batch takes them
  int32_t cap[4] = {0, 0, 0, 0};
  std::vector<float> packed[4];
  std::vector<int64_t> off[4];
  for (int k = 0; k < 4; ++k) {
    off[k].assign(P + 1, 0);
    for (int p = 0; p < P; ++p) {
      const int32_t n = (int32_t)(probs[p].cloud[k].size() / 4);
      cap[k] = n > cap[k] ? n : cap[k];
      off[k][p + 1] = off[k][p] + n;
      packed[k].insert(packed[k].end(), probs[p].cloud[k].begin(), probs[p].cloud[k].end());
    }
  }
  CHECK(llsr_scan2map_reserve(h, P, cap[2], cap[3], cap[0], cap[1]) == LLSR_OK, llsr_last_error(h));
  float* d_cloud[4];
  int64_t* d_off[4];
  for (int k = 0; k < 4; ++k) {
    CHECK(hipMalloc(&d_cloud[k], packed[k].size() * sizeof(float) + 16) == hipSuccess, "hipMalloc");
    CHECK(hipMalloc(&d_off[k], off[k].size() * sizeof(int64_t)) == hipSuccess, "hipMalloc");
    CHECK(hipMemcpy(d_cloud[k], packed[k].data(), packed[k].size() * sizeof(float), hipMemcpyHostToDevice) ==
              hipSuccess, "upload");
    CHECK(hipMemcpy(d_off[k], off[k].data(), off[k].size() * sizeof(int64_t), hipMemcpyHostToDevice) == hipSuccess,
          "upload");
  }
  std::vector<float> pose(6 * (size_t)P);
  for (int p = 0; p < P; ++p) std::memcpy(&pose[6 * (size_t)p], probs[p].pose, sizeof probs[p].pose);
  float* d_pose;
  llsr_lm_report* d_rep;
  int64_t* d_ne;
  CHECK(hipMalloc(&d_pose, pose.size() * sizeof(float)) == hipSuccess, "hipMalloc");
  CHECK(hipMalloc(&d_rep, P * sizeof(llsr_lm_report)) == hipSuccess, "hipMalloc");
  CHECK(hipMalloc(&d_ne, (size_t)P * LLSR_NE_WORDS * sizeof(int64_t)) == hipSuccess, "hipMalloc");
  CHECK(hipMemcpy(d_pose, pose.data(), pose.size() * sizeof(float), hipMemcpyHostToDevice) == hipSuccess, "upload");

  ncclUniqueId id;
  if (rank == 0) {
    CHECK(ncclGetUniqueId(&id) == ncclSuccess, "ncclGetUniqueId");
    if (world > 1) {
      const std::string tmp = id_file + ".tmp";
      std::ofstream f(tmp, std::ios::binary);
      f.write(reinterpret_cast<const char*>(&id), sizeof id);
      f.close();
      CHECK(std::rename(tmp.c_str(), id_file.c_str()) == 0, "publish the unique id");
    }
  } else {
    bool got = false;
    for (int k = 0; k < 600 && !got; ++k) {  // up to a minute
      std::ifstream f(id_file, std::ios::binary);
      if (f.good() && f.read(reinterpret_cast<char*>(&id), sizeof id)) got = true;
      else usleep(100000);
    }
    CHECK(got, "no unique id from rank 0");
  }
  ncclComm_t comm;
  CHECK(ncclCommInitRank(&comm, world, id, rank) == ncclSuccess, "ncclCommInitRank");
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess, "stream");

  llsr_s2m_batch b;
  std::memset(&b, 0, sizeof b);
  b.n_problems = P;
  b.corner_q = d_cloud[0]; b.corner_q_off = d_off[0];
  b.surf_q = d_cloud[1];   b.surf_q_off = d_off[1];
  b.corner_map = d_cloud[2]; b.corner_map_off = d_off[2];
  b.surf_map = d_cloud[3]; b.surf_map_off = d_off[3];
  b.pose = d_pose;
  b.report = d_rep;
  int32_t it = 0;
  const int32_t rc = llsr_scan2map_rccl(h, &b, comm, rank, world, d_ne, poll, &it, s);
  if (rc != LLSR_OK) {
    std::fprintf(stderr, "shard_driver: llsr_scan2map_rccl %d: %s / %s\n", rc, llsr_last_error(h),
                 ncclGetLastError(comm));
    return 1;
  }
  CHECK(hipStreamSynchronize(s) == hipSuccess, "sync");
  std::vector<llsr_lm_report> rep(P);
  CHECK(hipMemcpy(rep.data(), d_rep, P * sizeof(llsr_lm_report), hipMemcpyDeviceToHost) == hipSuccess, "download");
  float us = 0.0f;
  CHECK(llsr_rccl_allreduce_us(comm, d_ne, (int64_t)P * LLSR_NE_WORDS, 50, s, &us) == LLSR_OK, "allreduce probe");
  if (rank == 0) {
    std::ofstream out(argv[2], std::ios::binary);
    out.write(reinterpret_cast<const char*>(rep.data()), P * sizeof(llsr_lm_report));
    out.write(reinterpret_cast<const char*>(&us), sizeof us);
    out.write(reinterpret_cast<const char*>(&it), sizeof it);
    CHECK(out.good(), "write OUT");
  }
  std::printf("rank %d of %d: %d problems, %d LM iterations, allreduce %.2f us\n", rank, world, P, it, us);
  ncclCommDestroy(comm);
  (void)hipStreamDestroy(s);
  for (int k = 0; k < 4; ++k) {
    (void)hipFree(d_cloud[k]);
    (void)hipFree(d_off[k]);
  }
  (void)hipFree(d_pose);
  (void)hipFree(d_rep);
  (void)hipFree(d_ne);
  llsr_destroy(h);
  return 0;
}
