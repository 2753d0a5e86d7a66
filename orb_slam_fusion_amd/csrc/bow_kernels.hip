// gfx950 kernels of DBoW2's transform(features, BowVector&, FeatureVector&,
// levelsup) (3rdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1057-1179) over a
// vocabulary tree resident in HBM:
//
//   k_bow_descend   16 lanes per feature: at every level the lanes take the
//                   node's children (16 at a time), Hamming distance from 8
//                   v_bcnt, group minimum of (dist << 16 | child rank) = the
//                   reference's first strict minimum; stop at a node without
//                   children; word id, weight, and the node at depth
//                   L - levelsup
//   k_bow_assemble  block / frame: the std::map building of BowVector /
//                   FeatureVector: bitonic sort of (word, feature) and
//                   (node, feature) keys in LDS, per-word weight sums in
//                   feature order (addWeight) or first weight (addIfNotExist),
//                   the norm summed in word order by one lane, then the
//                   normalisation (BowVector.cpp:30-66, FeatureVector.cpp:28-38)
#include <hip/hip_runtime.h>

#include "lds_optin.h"
#include <stdint.h>

#include "bow_launch.h"

namespace orbgpu {

namespace {

constexpr uint64_t kNoKey = ~0ull;

__device__ __forceinline__ uint32_t group16_min(uint32_t v) {
#pragma unroll
  for (int off = 8; off >= 1; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off, 16));
  return v;
}

__global__ __launch_bounds__(256) void k_bow_descend(BowLaunch a) {
  const int f = blockIdx.y;
  const int i = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  const int n = a.n[f];
  const bool live = i < n;
  const size_t o = (size_t)f * a.stride + (live ? i : 0);
  const uint4* fd = reinterpret_cast<const uint4*>(a.descs + o * 32);
  const uint4 q0 = fd[0], q1 = fd[1];
  const VocabDev& V = a.voc;
  const int nid_level = V.L - a.levelsup;
  uint32_t node = 0, nid = 0;
  int level = 0;
  bool go = live;  // uniform over a feature's 16 lanes: shuffles stay in-group
  while (__builtin_amdgcn_ballot_w64(go) != 0) {
    if (go) {
      ++level;
      const int off = V.child_off[node], cnt = V.child_off[node + 1] - off;
      uint32_t best = 0xFFFFFFFFu;
      for (int j0 = 0; j0 < cnt; j0 += 16) {
        const int j = j0 + sub;
        if (j < cnt) {
          const uint32_t c = V.child_ids[off + j];
          const uint4* d = reinterpret_cast<const uint4*>(V.desc + (size_t)c * 32);
          const uint4 d0 = d[0], d1 = d[1];
          const uint32_t dist = __popc(d0.x ^ q0.x) + __popc(d0.y ^ q0.y) + __popc(d0.z ^ q0.z) +
                                __popc(d0.w ^ q0.w) + __popc(d1.x ^ q1.x) + __popc(d1.y ^ q1.y) +
                                __popc(d1.z ^ q1.z) + __popc(d1.w ^ q1.w);
          best = min(best, (dist << 16) | (uint32_t)j);
        }
      }
      best = group16_min(best);
      node = V.child_ids[off + (best & 0xFFFF)];
      if (level == nid_level) nid = node;
      go = V.child_off[node + 1] > V.child_off[node];
    }
  }
  if (live && sub == 0) {
    a.f_word[o] = V.word_id[node];
    a.f_weight[o] = V.weight[node];
    a.f_nid[o] = nid;
  }
}

// ascending bitonic sort of keys[0..m), m a power of two, whole block
__device__ void bitonic_sort(uint64_t* keys, int m) {
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < (m >> 1); t += blockDim.x) {
        const int lo = 2 * t - (t & (j - 1));  // index with bit j clear
        const int hi = lo + j;
        const bool up = (lo & k) == 0;
        const uint64_t x = keys[lo], y = keys[hi];
        if ((x > y) == up) keys[lo] = y, keys[hi] = x;
      }
      __syncthreads();
    }
  }
}

// exclusive scan of one int per thread over the 256-thread block; returns the
// thread's offset, *total the sum (tmp: 4 ints of LDS)
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) tmp[w] = inc;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < w; ++i) base += tmp[i];
  *total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
  __syncthreads();
  return base + inc - v;
}

// keys: m u64, fw: m doubles (dynamic LDS)
__global__ __launch_bounds__(256) void k_bow_assemble(BowLaunch a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t bow_lds[];
  __shared__ int tmp[4];
  __shared__ double norm_s;
  const int f = blockIdx.x, t = threadIdx.x;
  const int n = a.n[f];
  const size_t o = (size_t)f * a.stride;
  int m = 1;
  while (m < n) m <<= 1;
  uint64_t* keys = reinterpret_cast<uint64_t*>(bow_lds);
  double* fw = reinterpret_cast<double*>(bow_lds + 8 * (size_t)a.lds_m);
  const VocabDev& V = a.voc;
  const bool tf = V.weighting == 0 || V.weighting == 1;
  const bool must = V.scoring != 5;
  const bool empty = V.n_words == 0;
  // ---- BowVector
  for (int i = t; i < m; i += 256) {
    uint64_t k = kNoKey;
    if (i < n) {
      const double w = a.f_weight[o + i];
      fw[i] = w;
      if (!empty && w > 0) k = ((uint64_t)a.f_word[o + i] << 32) | (uint32_t)i;
    }
    keys[i] = k;
  }
  __syncthreads();
  bitonic_sort(keys, m);
  // segment heads -> output slots
  const int per = (m + 255) / 256;
  const int b = min(t * per, m), e = min(b + per, m);
  auto head = [&](int i) {
    return keys[i] != kNoKey && (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32));
  };
  int cnt = 0;
  for (int i = b; i < e; ++i) cnt += head(i);
  int n_words;
  int pos = block_excl_scan(cnt, tmp, &n_words);
  uint32_t* bw = a.bow_words + o;
  double* bwt = a.bow_weights + o;
  double wsum[32];  // per <= 32 (m <= kBowMaxFeatures = 8192)
  int nh = 0;
  for (int i = b; i < e; ++i) {
    if (!head(i)) continue;
    double w = fw[(uint32_t)keys[i]];
    if (tf) {  // addWeight: the later features of the word, in feature order
      const uint64_t word = keys[i] >> 32;
      for (int j = i + 1; j < m && keys[j] != kNoKey && (keys[j] >> 32) == word; ++j)
        w += fw[(uint32_t)keys[j]];
    }
    bw[pos + nh] = (uint32_t)(keys[i] >> 32);
    wsum[nh++] = w;
  }
  __syncthreads();  // fw no longer read: it now holds the word weights in word order
  for (int h = 0; h < nh; ++h) fw[pos + h] = wsum[h];
  __syncthreads();
  if (must) {
    if (t == 0) {  // BowVector::normalize: summed in word order, one chain
      double norm = 0.0;
      int i = 0;
      if (V.scoring == 1) {
        for (; i + 8 <= n_words; i += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = fw[i + u];
#pragma unroll
          for (int u = 0; u < 8; ++u) norm = __builtin_fma(v[u], v[u], norm);
        }
        for (; i < n_words; ++i) norm = __builtin_fma(fw[i], fw[i], norm);
        norm = sqrt(norm);
      } else {
        for (; i + 8 <= n_words; i += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = fw[i + u];
#pragma unroll
          for (int u = 0; u < 8; ++u) norm += fabs(v[u]);
        }
        for (; i < n_words; ++i) norm += fabs(fw[i]);
      }
      norm_s = norm;
    }
    __syncthreads();
    const double norm = norm_s;
    for (int i = t; i < n_words; i += 256) bwt[i] = norm > 0.0 ? fw[i] / norm : fw[i];
  } else {
    const double nd = (double)n_words;
    for (int i = t; i < n_words; i += 256) bwt[i] = tf ? fw[i] / nd : fw[i];
  }
  __syncthreads();
  // ---- FeatureVector
  for (int i = t; i < m; i += 256) {
    uint64_t k = kNoKey;
    if (i < n && !empty && a.f_weight[o + i] > 0) k = ((uint64_t)a.f_nid[o + i] << 32) | (uint32_t)i;
    keys[i] = k;
  }
  __syncthreads();
  bitonic_sort(keys, m);
  cnt = 0;
  int kept = 0;
  for (int i = b; i < e; ++i) {
    cnt += head(i);
    kept += keys[i] != kNoKey;
  }
  int n_nodes, n_kept;
  pos = block_excl_scan(cnt, tmp, &n_nodes);
  (void)block_excl_scan(kept, tmp, &n_kept);
  uint32_t* fn = a.fv_nodes + o;
  int32_t* fo = a.fv_offsets + (size_t)f * (a.stride + 1);
  uint32_t* ff = a.fv_features + o;
  for (int i = b; i < e; ++i) {
    if (keys[i] == kNoKey) continue;
    ff[i] = (uint32_t)keys[i];  // sorted position = output position
    if (head(i)) {
      fn[pos] = (uint32_t)(keys[i] >> 32);
      fo[pos] = i;
      ++pos;
    }
  }
  if (t == 0) {
    fo[n_nodes] = n_kept;
    a.n_words[f] = n_words;
    a.n_nodes[f] = n_nodes;
  }
}

}  // namespace

hipError_t launch_bow(const BowLaunch& a, hipStream_t st) {
  if (a.n_frames <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bow_descend, dim3((unsigned)((a.stride + 15) / 16), a.n_frames), dim3(256),
                     0, st, a);
  const size_t lds = 16 * (size_t)a.lds_m;
  if (lds > 64 * 1024) {
    if (lds_optin(reinterpret_cast<const void*>(&k_bow_assemble), 16 * kBowMaxFeatures) != hipSuccess)
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(k_bow_assemble, dim3(a.n_frames), dim3(256), lds, st, a);
  return hipGetLastError();
}

}  // namespace orbgpu
