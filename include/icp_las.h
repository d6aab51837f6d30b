/*
 * icp_las.h — LAS 1.2 point I/O of the two reference front-ends (host only, no GPU):
 *   icp_las_read        LASIO::readLAS (core/lasio.cpp:7-125; signature check, maxPoints
 *                       truncation) and readLASFile (icp_registration.cpp:248-378; rejects 0 or
 *                       > 1e8 points) — x = X * scale + offset per axis
 *   icp_las_write_core  LASIO::writeLAS (core/lasio.cpp:127-210): scale 0.001, offset = min
 *   icp_las_write_cli   saveResultAsLAS (icp_registration.cpp:698-815): caller's scale/offset
 *   icp_write_transform_report  saveTransformation (icp_registration.cpp:625-695), same text
 * Integer conversion truncates toward zero, as the reference's casts do.
 */
#ifndef ICP_LAS_H
#define ICP_LAS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ICP_LAS_CORE 0 /* LASIO::readLAS rules   */
#define ICP_LAS_CLI 1  /* readLASFile rules      */

typedef struct icp_las_header {
  uint32_t offset_to_points;
  uint32_t num_points;
  uint16_t record_length;
  double scale[3];
  double offset[3];
  double max[3];
  double min[3];
} icp_las_header;

/* Header only. Returns 0 on success, -1 if the file cannot be opened/read, -2 bad signature
 * (core rules) or bad point count (CLI rules). */
int icp_las_read_header(const char* path, int rules, icp_las_header* hdr);

/* Points (AoS xyz). xyz_out must hold min(num_points, max_points) points (max_points 0 = all;
 * with CLI rules, whose reader has no limit, max_points only bounds the output buffer).
 * Returns the number of points read (>= 0) or a negative error as above. */
int64_t icp_las_read(const char* path, int rules, int64_t max_points, double* xyz_out, icp_las_header* hdr);

/* LASIO::writeLAS with the bounds of the given points (PointCloud::computeBounds first). */
int icp_las_write_core(const char* path, const double* xyz, int64_t n);
/* LASIO::writeLAS with the caller's PointCloud bounds as they stand (minX, maxX, minY, maxY, minZ,
 * maxZ): the writer's offset is minX/minY/minZ whatever the points are now. The reference service
 * saves the registered source with the bounds computed when it was loaded
 * (registrationservice.cpp:98, :156), so its coordinates can fall below the offset. */
int icp_las_write_core_bounds(const char* path, const double* xyz, int64_t n, const double bounds[6]);
int icp_las_write_cli(const char* path, const double* xyz, int64_t n, const double scale[3], const double offset[3]);

/* R row-major 3x3, t[3]; transforms: n_transforms cumulative 4x4 (row-major) or null. */
int icp_write_transform_report(const char* path, const double R[9], const double t[3], const double* transforms,
                               int32_t n_transforms);

#ifdef __cplusplus
}
#endif
#endif
