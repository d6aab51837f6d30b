// query_order.h — spatially compact order of the source queries (see query_order.cpp).
#pragma once

#include <cstdint>
#include <vector>

namespace icp {

// perm[k] = caller index of the query placed at slot k.
void kd_query_order(const double* xyz, int64_t n, int bucket, std::vector<int32_t>* perm);

}  // namespace icp
