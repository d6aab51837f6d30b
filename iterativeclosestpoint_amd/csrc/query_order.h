// query_order.h — spatially compact order of the source queries (see query_order.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace icp {

// perm[k] = caller index of the query placed at slot k.
void kd_query_order(const double* xyz, int64_t n, int bucket, std::vector<int32_t>* perm);

// The same partition built on the device from the AoS cloud in HBM (query_order_gpu.hip):
// d_perm[k] = cloud index of slot k. Synchronises the stream.
hipError_t gpu_kd_query_order(const double* d_xyz, int64_t n, int bucket, int32_t* d_perm, hipStream_t s);

}  // namespace icp
