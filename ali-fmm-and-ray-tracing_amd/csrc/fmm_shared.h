// fmm_shared.h — host/device structs shared by the FMM kernels and the C-ABI host code.
#pragma once
#include <stdint.h>

namespace af {

// per-source job of the exact-heap initialisation kernel (travel(), subgrid 1)
struct InitJob {
  long isx, isz;  // source node (round((scx-gox)/dnx), :1509-1510)
  double dnx, dnz;
  int exact_r;    // radius [nodes] of the exact heap-ordered main-loop prefix (0: none)
  double tstop;   // = exact_r * dnx / vmax
};

// nodes handed to the main grid: decimated stage 3 (<= 27 x 27) or the exact prefix window
constexpr int kHandoverMax = 109 * 109;
struct HandoverOut {
  int n;
  int err;
  int cell[kHandoverMax];
  double ttn[kHandoverMax];
  signed char cls[kHandoverMax];  // 1 known inner, 2 known outer (-> close), 3 close
  // profile (wall-clock 100 MHz ticks): [0..3] stage 1, 2, 3, main prefix; [4..7] their pops;
  // [8..11] relax-role busy ticks per stage; [12..15] relaxations | evaluation passes << 24 | fouds18_A() fallbacks << 44
  long long prof[16];
};

// status codes of the band kernel (valid for update() = st >= 0; known for fouds18 = st == 0)
enum : int { kFar = -1, kFarCand = -3, kKnown = 0, kClose = 1, kCloseCand = 2 };

}  // namespace af
