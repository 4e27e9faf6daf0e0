// Internal to the K2 probe sources (hdp_probe.hip: split / sweep paths, planning, native queue;
// hdp_probe_team.hip: the single-read team path).  Not part of the C-ABI.
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
  float* slabH;     // split / sweep: [ksh][T][rp];  team: X side partials [S][ksh][16][rp]
  float* slabJ;     // split / sweep: [ksj][T][rp];  team: G side partials [S][ksj][16][rp]
  float* partA;     // [kst][rp][in]
  float* partB;     // [kst][out][rp]
  float* yH;        // sweep: H = X A^T [T][rp];  team: X side projection granules [S][16][rp] (8 B)
  float* yJ;        // sweep: J = G B   [T][rp];  team: G side projection granules
  int64_t T, in, out;
  float scale;
  int r, b_t, accumulate;
  int ksh, ksj, kst;
  int colh, colj;   // P1 columns per wave (multiples of 16)
  int ldb;          // row stride of gB: r, or the module's full rank when this is one of its r-slices
};

// a group as planned on the host (sweep / team paths: any size, descriptors uploaded per flush)
struct HostGroup {
  int n = 0, rp = 16, RB = 1;
  std::vector<ProbeDesc> d;
};

constexpr int kTileLd = 72;          // padded LDS row (floats) of the PROJ transpose tiles
constexpr int kSwWaves = 8;          // streaming waves of a sweep / team workgroup
constexpr int kSwC = 64 * kSwWaves;  // stripe width (columns)

// pinned staging ring -> device table region, stream-ordered (hdp_probe.hip)
int probe_tables_upload(const std::vector<char>& blob, void* dst, hipStream_t st);

// team path (hdp_probe_team.hip)
// bytes of the group-level team tables (sides, item lists) for n modules
size_t team_table_bytes(int n);
size_t team_table_per_module();
// workgroups one team launch uses (one per CU) and whether every module's team fits in it
int team_grid();
bool team_fits(const HostGroup& ga);
// launch the team kernel over the group; `tab` = the group's table region (team_table_bytes),
// `cnt` = the group's contiguous counter block of `cnt_bytes` (zeroed here, stream-ordered)
int launch_team(const HostGroup& ga, int x_dtype, char* tab, int* cnt, size_t cnt_bytes, hipStream_t st);
// the device error word of the team path (a bounded exchange wait gave up): read + clear
int team_errors(int clear);

}  // namespace hdp
