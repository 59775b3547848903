// bmqcrc_internal.h -- shared between the host dispatcher and the HIP kernels.
#pragma once
#include <stdint.h>

namespace bmqcrc {

// One wave owns 64 segments; per round each segment advances one 128-byte
// line (= 32 dwords = one full turn of the 32-word fold ring).
constexpr int kLine = 128;
constexpr int kWaveLanes = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kSlots = 2;                                  // LDS ring depth per wave
constexpr int kSlotBytes = kWaveLanes * kLine;             // 8 KiB per round per wave
constexpr int kLdsBytes = kWavesPerBlock * kSlots * kSlotBytes;  // 64 KiB per block
constexpr int kTabBytes = 8 * 256 * 4;  // remainder-reduction slicing tables (LDS)
constexpr uint32_t kDefaultSegBytes = 16384;
constexpr int kPlanBlock = 1024;

// Control words written by the planner (device memory, 4 x u32).
//   [0] total segments   [1] 1 if every message is exactly one segment
//   [2] number of 64-segment groups
struct PlanCtrl {
    uint32_t total_segs;
    uint32_t identity;
    uint32_t ngroups;
    uint32_t pad;
};

struct BatchArgs {
    const uint8_t* arena;      // device
    const uint64_t* offsets;   // device, n
    const uint32_t* lengths;   // device, n
    const uint32_t* seeds;     // device, n, or nullptr (all zero)
    uint32_t* out;             // device, n
    uint32_t* seg_first;       // workspace, n (exclusive prefix of segment counts)
    uint32_t* block_sum;       // workspace, 2 * nblocks
    uint32_t* seg2msg;         // workspace, max_segs
    PlanCtrl* ctrl;            // workspace
    uint64_t n;
    uint32_t seg_bytes;
    uint32_t nblocks;          // planner blocks = ceil(n / kPlanBlock)
    uint64_t max_segs;
    uint32_t tune;             // experiment knobs (BMQCRC_TUNE env): bit0 disables nt LDS-DMA
                               // loads, bit1 selects a 1-block/CU grid
    uint32_t pad;
};

}  // namespace bmqcrc

// Launchers (crc32c_kernels.hip).  All asynchronous on `stream`.
extern "C" int bmqcrc_launch_batch(const bmqcrc::BatchArgs* a, void* stream, int num_cus,
                                   void* ev_start, void* ev_stop);
extern "C" int bmqcrc_launch_fill(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t begin,
                                  void* stream);
