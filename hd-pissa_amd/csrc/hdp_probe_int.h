// Internal to the K2 probe source (hdp_probe.hip: split / sweep paths, planning, native queue).
// Not part of the C-ABI.
#pragma once

#include <vector>

#include "hdp_common.h"

namespace hdp {

// one module of a probe group as the host plans it (pointers into the caller's tensors and the
// group workspace)
struct ProbeDesc {
  const void* X;
  const void* G;
  const float* A;
  const float* B;   // B (out x r) or B^T (r x out) when b_t
  float* gA;
  float* gB;
  float* slabH;     // split / sweep: [ksh][T][rp]
  float* slabJ;     // split / sweep: [ksj][T][rp]
  float* partA;     // [kst][rp][in]
  float* partB;     // [kst][out][rp]
  float* yH;        // sweep: H = X A^T [T][rp]
  float* yJ;        // sweep: J = G B   [T][rp]
  int64_t T, in, out;
  float scale;
  int r, b_t, accumulate;
  int ksh, ksj, kst;
  int colh, colj;   // P1 columns per wave (multiples of 16)
  int ldb;          // row stride of gB: r, or the module's full rank when this is one of its r-slices
};

// a group as planned on the host (sweep path: any size, descriptors uploaded per flush)
struct HostGroup {
  int n = 0, rp = 16, RB = 1;
  std::vector<ProbeDesc> d;
};

constexpr int kTileLd = 72;          // padded LDS row (floats) of the PROJ transpose tiles
constexpr int kSwWaves = 8;          // streaming waves of a sweep workgroup
constexpr int kSwC = 64 * kSwWaves;  // stripe width (columns)

// pinned staging ring -> device table region, stream-ordered (hdp_probe.hip)
int probe_tables_upload(const std::vector<char>& blob, void* dst, hipStream_t st);

}  // namespace hdp
