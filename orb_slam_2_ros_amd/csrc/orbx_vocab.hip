// orbx_vocab.hip -- DBoW2 vocabulary transform on gfx950: the descent of
// TemplatedVocabulary::transform(feature, word, weight, nid, levelsup)
// (TemplatedVocabulary.h:1231-1272) for every feature of a frame (or batch).
//
// A group of G lanes (G >= the branching factor k: 16 for ORBvoc's k = 10)
// takes one feature.  At each level lane c loads child c's descriptor; the
// children of a node sit in consecutive slots, so a group reads one
// contiguous run of 32-B rows.  The Hamming distances are reduced to the first
// minimum (the reference's `d < best_d` over children in order) with DPP row
// operations, and the group moves to that child, until a node without
// children.  The node at level L - levelsup is the FeatureVector node.
#include <hip/hip_runtime.h>

#include "orbx_device.h"
#include "orbx_wave.h"

namespace orbx {
namespace {

constexpr int kVT = 256;
constexpr uint32_t kNoNode = 0xFFFFFFFFu;

__device__ inline int hamming_rr(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Minimum over each group of G consecutive lanes (G = 16, 32 or 64), in every
// lane of the group.  Whole wave active.
template <int G>
__device__ inline uint32_t group_min(uint32_t v, int lane) {
    v = min(v, dpp_or<kRowShr1>(~0u, v));
    v = min(v, dpp_or<kRowShr2>(~0u, v));
    v = min(v, dpp_or<kRowShr4>(~0u, v));
    v = min(v, dpp_or<kRowShr8>(~0u, v));   // lane 15 of each row: the row minimum
    uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    if (G >= 32) { r0 = r1 = min(r0, r1); r2 = r3 = min(r2, r3); }
    if (G >= 64) { r0 = r1 = r2 = r3 = min(r0, r2); }
    const int row = lane >> 4;
    return row == 0 ? r0 : row == 1 ? r1 : row == 2 ? r2 : r3;
}

template <int G>
__global__ __launch_bounds__(kVT) void k_vocab_transform(VocabDev v, const uint8_t *feat, int n, int nid_level,
                                                         uint32_t *o_word, double *o_weight, uint32_t *o_node) {
    const int lane = threadIdx.x & 63, c = lane & (G - 1);
    const int f = (int)((blockIdx.x * (unsigned)kVT + threadIdx.x) / G);
    const bool active = f < n;
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
    if (active) {
        const uint4 *fp = reinterpret_cast<const uint4 *>(feat + 32 * (int64_t)f);
        q0 = fp[0]; q1 = fp[1];
    }
    int slot = 0, level = 0;
    uint32_t nid = nid_level <= 0 ? 0u : kNoNode;
    VocabNode nd = v.nodes[0];
    while (true) {
        const bool going = active && nd.nchild > 0;
        if (__ballot(going) == 0) break;
        uint32_t key = ~0u;
        if (going && c < nd.nchild) {
            const uint4 *dp = reinterpret_cast<const uint4 *>(v.desc + 32 * (int64_t)(nd.first + c));
            key = ((uint32_t)hamming_rr(q0, q1, dp[0], dp[1]) << 8) | (uint32_t)c;
        }
        const uint32_t m = group_min<G>(key, lane);
        if (going) {
            slot = nd.first + (int)(m & 0xFF);
            nd = v.nodes[slot];
            if (++level == nid_level) nid = nd.id;
        }
    }
    if (active && c == 0) {
        o_word[f] = nd.word;
        o_weight[f] = v.weight[slot];
        // a leaf above level L - levelsup: the reference leaves nid unset (UB); the leaf here
        o_node[f] = nid == kNoNode ? nd.id : nid;
    }
}

}  // namespace

hipError_t launch_vocab_transform(const VocabDev &v, const uint8_t *feat, int n, int nid_level, uint32_t *o_word,
                                  double *o_weight, uint32_t *o_node, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (v.k <= 16) {
        const int per = kVT / 16;
        hipLaunchKernelGGL(k_vocab_transform<16>, dim3((n + per - 1) / per), dim3(kVT), 0, st, v, feat, n, nid_level,
                           o_word, o_weight, o_node);
    } else if (v.k <= 32) {
        const int per = kVT / 32;
        hipLaunchKernelGGL(k_vocab_transform<32>, dim3((n + per - 1) / per), dim3(kVT), 0, st, v, feat, n, nid_level,
                           o_word, o_weight, o_node);
    } else if (v.k <= 64) {
        const int per = kVT / 64;
        hipLaunchKernelGGL(k_vocab_transform<64>, dim3((n + per - 1) / per), dim3(kVT), 0, st, v, feat, n, nid_level,
                           o_word, o_weight, o_node);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace orbx
