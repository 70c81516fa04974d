// The stream aggregation kernels (k_update_mixed<256>, and k_update_encode<256>, the
// headline step) in a translation unit of their own, so that fleet_amd/build.py can
// compile them with the ILP-first machine scheduler: they are VALU-issue bound at 5-6
// waves per SIMD, where it beats the default occupancy-first scheduler, while the
// tiled and pipelined kernels of kernels.hip lose under it (DESIGN.md §4.1,
// profiles/r02/sched_ilp_ab.txt).
#define FLEET_STREAM_TU
#include "kernels.hip"
