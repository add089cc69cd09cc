// masks.hip — token-level loss / response masks and score placement (gfx950).
//
//  rmi_masks_and_scores   get_masks_and_scores (ctx_manager.py:35-70)
//
// One wave per row streams the row's token ids in chunks of 256 (4 consecutive ids per lane,
// 32-B loads; the loads of 8 chunks are issued together): turn = cumsum(ids == <|im_start|>)
// is a DPP wave prefix scan per chunk plus a running carry, the masks are written as they are produced ([:, :-1] slice), the score row
// is zero-filled in the same pass ([:, 1:] slice), and the reward-token positions of each
// assistant turn are recorded in LDS.  After the pass (stores fenced) the <= 64 turn scores
// are scattered to their positions (Qwen: rolled by +1) — exactly the boolean-mask
// assignment order of the reference, including its fallback to the last column.
// Algorithmic traffic: 8 B/token in, 6 B/token out.
#include "common.hpp"

namespace rmi {
namespace {

constexpr int kMaxSlots = 64;  // turn slots (zip_longest length) handled per row
constexpr int kTok = 4;        // token ids per lane per chunk
constexpr int kChunk = 64 * kTok;

struct __attribute__((packed, aligned(8))) I64x4 {
  int64_t a, b, c, d;
};
struct __attribute__((packed, aligned(1))) U32u {
  uint32_t x;
};
struct __attribute__((packed, aligned(4))) F4u {
  float x, y, z, w;
};

// 32 readable bytes for the clamped loads of groups outside a row's tokens
__device__ const int64_t kZero4[kTok] = {0, 0, 0, 0};

constexpr int kSuper = 8;  // chunks whose loads are issued together (2048 ids per row)

// The batch assembly of formulate_rollouts (ctx_manager.py:278-306) fused into the same pass
// (kAsm): row b of the left-padded batch is pad_id * (S - n_b) followed by the row's n_b
// tokens tokens[off[b] .. off[b+1]); the pass writes input_ids, attention_mask (1 on the
// tokens) and position_ids = cumsum(attention_mask) next to the masks and scores.
struct AsmArgs {
  const int64_t* tokens;
  const int64_t* off;     // row b = tokens[off[b] .. off[b+1]), or with len: tokens[off[b] .. off[b] + len[b])
  const int32_t* len;
  int64_t pad_id;
  int64_t* input_ids;
  int64_t* attention_mask;
  int64_t* position_ids;
  int32_t* resp_count;     // (optional) per row: the response_mask ones written (response_length)
  const float* last_score;  // (optional, no turn scores) score[:, -1] = last_score[b]: the normalised score
};

template <bool kAsm>
__global__ __launch_bounds__(64) void masks_kernel(const int64_t* __restrict__ ids, int64_t B, int64_t S, int64_t sp,
                                                   int64_t rt, const double* __restrict__ scores,
                                                   const int32_t* __restrict__ n_scores, int T, int n_slots,
                                                   int flags, float* __restrict__ score_out,
                                                   uint8_t* __restrict__ lmask, uint8_t* __restrict__ rmask,
                                                   uint8_t* __restrict__ err, AsmArgs as) {
  __shared__ int pos[kMaxSlots], cnt[kMaxSlots];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  pos[lane] = -1;
  cnt[lane] = 0;
  __syncthreads();
  const int64_t So = S - 1;  // output columns
  const int64_t* row = kAsm ? nullptr : ids + b * S;
  int64_t a_src = 0, pad = 0;
  uint8_t e_unsup = 0;  // the row's error byte is written once, at the end (no pre-zeroed buffer)
  if (kAsm) {
    const int64_t o0 = as.off[b], o1 = as.len ? o0 + as.len[b] : as.off[b + 1];
    pad = S - (o1 - o0);
    if (pad < 0) {  // a row longer than S: flagged, assembled from its last S tokens
      e_unsup = RMI_ERR_UNSUP;
      a_src = o1 - S;
      pad = 0;
    } else {
      a_src = o0 - pad;  // column p holds tokens[a_src + p] for p >= pad
    }
  }
  float* srow = score_out + b * So;
  uint8_t* lrow = lmask + b * So;
  uint8_t* rrow = rmask + b * So;
  const bool turn_scores = flags & RMI_MS_TURN_SCORES, resp_only = flags & RMI_MS_RESPONSE_MASK;
  // an id matching neither special token, for positions past the row end
  const int64_t none = (sp != -1 && rt != -1) ? -1 : ((sp != -2 && rt != -2) ? -2 : -3);
  int carry = 0;
  int n_resp = 0;  // response_mask ones of the row (kAsm with resp_count)
  for (int64_t s0 = 0; s0 < S; s0 += kSuper * kChunk) {
    // 1. every load of the super-chunk in flight together (clamped addresses, branch-free);
    //    the group at the row end and groups past it are fixed up element-wise afterwards
    I64x4 v[kSuper];
    if (kAsm) {  // padded ids from the ragged rows: 32-B loads where the group lies inside the
                 // row's tokens (clamped to a zero block elsewhere), element-wise fix-up after
#pragma unroll
      for (int k = 0; k < kSuper; ++k) {
        const int64_t p0 = s0 + k * kChunk + kTok * lane;
        const bool full = p0 >= pad && p0 + kTok <= S;
        v[k] = *reinterpret_cast<const I64x4*>(full ? as.tokens + a_src + p0 : kZero4);
      }
#pragma unroll
      for (int k = 0; k < kSuper; ++k) {
        const int64_t p0 = s0 + k * kChunk + kTok * lane;
        if (!(p0 >= pad && p0 + kTok <= S)) {  // the pad, the pad / token edge and the row end
          int64_t e4[kTok];
#pragma unroll
          for (int e = 0; e < kTok; ++e) {
            const int64_t p = p0 + e;
            e4[e] = p >= S ? none : (p < pad ? as.pad_id : as.tokens[a_src + p]);
          }
          v[k] = I64x4{e4[0], e4[1], e4[2], e4[3]};
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < kSuper; ++k) {
        const int64_t p0 = s0 + k * kChunk + kTok * lane;
        v[k] = *reinterpret_cast<const I64x4*>(row + (p0 + kTok <= S ? p0 : 0));
      }
    }
    if (!kAsm && s0 + kSuper * kChunk > S) {
#pragma unroll
      for (int k = 0; k < kSuper; ++k) {
        const int64_t p0 = s0 + k * kChunk + kTok * lane;
        if (p0 + kTok > S) {
          int64_t e4[kTok];
          for (int e = 0; e < kTok; ++e) e4[e] = p0 + e < S ? row[p0 + e] : none;
          v[k] = I64x4{e4[0], e4[1], e4[2], e4[3]};
        }
      }
    }
    // 2. per chunk: turn prefix scan, masks, zero fill, reward positions
#pragma unroll
    for (int k = 0; k < kSuper; ++k) {
      const int64_t p0 = s0 + k * kChunk + kTok * lane;
      if (s0 + k * kChunk >= S) break;  // wave-uniform
      const int64_t t[kTok] = {v[k].a, v[k].b, v[k].c, v[k].d};
      if (kAsm) {  // input_ids, attention_mask, position_ids of the padded row
        int64_t* io = as.input_ids + b * S;
        int64_t* ao = as.attention_mask + b * S;
        int64_t* po = as.position_ids + b * S;
        int64_t am[kTok], ps[kTok];
#pragma unroll
        for (int e = 0; e < kTok; ++e) {
          const int64_t p = p0 + e;
          am[e] = p >= pad ? 1 : 0;
          ps[e] = p >= pad ? p - pad + 1 : 0;
        }
        if (p0 + kTok <= S) {  // 32-B stores
          *reinterpret_cast<I64x4*>(io + p0) = v[k];
          *reinterpret_cast<I64x4*>(ao + p0) = I64x4{am[0], am[1], am[2], am[3]};
          *reinterpret_cast<I64x4*>(po + p0) = I64x4{ps[0], ps[1], ps[2], ps[3]};
        } else {
#pragma unroll
          for (int e = 0; e < kTok; ++e)
            if (p0 + e < S) {
              io[p0 + e] = t[e];
              ao[p0 + e] = am[e];
              po[p0 + e] = ps[e];
            }
        }
      }
      int st[kTok], c = 0;
#pragma unroll
      for (int e = 0; e < kTok; ++e) {
        st[e] = t[e] == sp;
        c += st[e];
      }
      const int incl = wave_inclusive_scan(c);
      int turn = carry + incl - c;
      carry += __builtin_amdgcn_readlane(incl, 63);
      uint32_t lm = 0, rm = 0;
#pragma unroll
      for (int e = 0; e < kTok; ++e) {
        turn += st[e];  // turn_indicators at p0 + e
        const uint32_t r = (turn & 1) && turn > 1;
        const uint32_t l = resp_only ? r : (uint32_t)(turn > 1);
        rm |= r << (8 * e);
        lm |= l << (8 * e);
        if (turn_scores && t[e] == rt && (turn & 1) && turn >= 3) {
          const int idx = (turn - 3) >> 1;  // turn_indicator = idx * 2 + 3
          if (idx < n_slots) {
            atomicAdd(&cnt[idx], 1);
            pos[idx] = (int)(p0 + e);
          }
        }
      }
      // masks[:, :-1]: columns p < S - 1
      if (kAsm && as.resp_count)
        n_resp += __builtin_popcount(p0 + kTok <= So ? rm : (p0 >= So ? 0u : rm & ((1u << (8 * (So - p0))) - 1u)));
      if (p0 + kTok <= So) {
        reinterpret_cast<U32u*>(lrow + p0)->x = lm;
        reinterpret_cast<U32u*>(rrow + p0)->x = rm;
      } else {
#pragma unroll
        for (int e = 0; e < kTok; ++e)
          if (p0 + e < So) {
            lrow[p0 + e] = (uint8_t)(lm >> (8 * e));
            rrow[p0 + e] = (uint8_t)(rm >> (8 * e));
          }
      }
      // score[:, 1:] zero fill: output column p - 1 for p in [1, S)
      if (p0 >= 1 && p0 + kTok <= S) {
        *reinterpret_cast<F4u*>(srow + p0 - 1) = F4u{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int e = 0; e < kTok; ++e)
          if (p0 + e >= 1 && p0 + e < S) srow[p0 + e - 1] = 0.f;
      }
    }
  }
  // the zero fill has completed (this wave's stores retired) before the scattered scores land
  // on it, and the LDS position records are visible to every lane: a plain counter wait —
  // a __threadfence() here would add an L2 write-back per row
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (kAsm && as.resp_count) {
    for (int o = 32; o > 0; o >>= 1) n_resp += __shfl_xor(n_resp, o, 64);
    if (lane == 0) as.resp_count[b] = n_resp;
  }
  if (So <= 0 || !turn_scores) {  // no per-turn positions: only the overlong bit can be set
    if (lane == 0) err[b] = e_unsup;
  }
  if (So <= 0) return;  // a one-column batch has no score / mask columns
  if (!turn_scores) {
    if (lane == 0) {  // score_tensor[:, -1] = python sum(all_scores[b]), kept by [:, 1:]
      if (kAsm && as.last_score) {  // (normalised already: _normalize_score_tensor in place)
        srow[So - 1] = as.last_score[b];
      } else {
        double sum = 0.0;
        for (int i = 0; i < n_scores[b]; ++i) sum += scores[(int64_t)i * B + b];
        srow[So - 1] = (float)sum;
      }
    }
    return;
  }
  const bool roll = flags & RMI_MS_ROLL;
  const int nb = n_scores[b];
  const bool slot = lane < n_slots;
  const float s = slot && lane < nb && lane < T ? (float)scores[(int64_t)lane * B + b] : 0.0f;
  const int n = slot ? cnt[lane] : 0, p = slot ? pos[lane] : -1;
  // the reference's mask assignment raises on a turn with several reward positions
  const bool multi = __any(n > 1);  // (a wave-wide vote: every lane takes part)
  if (lane == 0) err[b] = e_unsup | (multi ? (uint8_t)RMI_ERR_STATE : (uint8_t)0);
  // positions -> output column: roll (+1, Qwen) then drop column 0
  auto out_col = [&](int64_t q) -> int64_t { return (roll ? (q + 1) % S : q) - 1; };
  if (slot && n == 1 && p != S - 1) {
    const int64_t o = out_col(p);
    if (o >= 0) srow[o] = s;
  }
  // the last column: written by every slot without a position (fallback) or positioned there,
  // the largest such slot last
  const uint64_t last = __ballot(slot && (n == 0 || p == S - 1));
  if (last) {
    const int hi = 63 - __clzll(last);
    if (lane == hi) {
      const int64_t o = out_col(S - 1);
      if (o >= 0) srow[o] = s;
    }
  }
}

// per-row count of the nonzero bytes of a u8 [B, S] mask (response_mask.sum(-1)): a wave per
// row, dword loads where the row is 4-B aligned, a wave reduction
__global__ __launch_bounds__(256) void row_counts_kernel(const uint8_t* __restrict__ m, int64_t B, int64_t S,
                                                         int32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= B) return;
  const uint8_t* row = m + i * S;
  int c = 0;
  int64_t k0 = 0;
  if ((S & 3) == 0) {  // every row 4-B aligned (the base is): whole dwords
    const uint32_t* w = reinterpret_cast<const uint32_t*>(row);
    for (int64_t k = lane; k < (S >> 2); k += 64) {
      const uint32_t x = w[k];
      c += ((x & 0xFFu) != 0) + ((x & 0xFF00u) != 0) + ((x & 0xFF0000u) != 0) + ((x >> 24) != 0);
    }
    k0 = S;
  }
  for (int64_t k = k0 + lane; k < S; k += 64) c += row[k] != 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) out[i] = c;
}

}  // namespace
}  // namespace rmi

RMI_API int rmi_row_counts(const uint8_t* mask, int64_t B, int64_t S, int32_t* out, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || S < 0 || (B > 0 && (!out || (S > 0 && !mask)))) return RMI_EINVAL;
  if (B > 0x7FFFFFFFll * 4) return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if ((S & 3) == 0 && (reinterpret_cast<uintptr_t>(mask) & 3u)) return RMI_EUNSUP;
  hipLaunchKernelGGL(row_counts_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, as_stream(stream), mask, B, S,
                     out);
  return launch_status();
}

RMI_API int rmi_masks_and_scores(const int64_t* ids, int64_t B, int64_t S, int64_t special_token,
                                 int64_t reward_token, const double* scores, const int32_t* n_scores, int32_t T,
                                 int32_t n_slots, int32_t flags, float* score_out, uint8_t* loss_mask,
                                 uint8_t* response_mask, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || S < 0 || T < 0 || n_slots < 0) return RMI_EINVAL;
  if (n_slots > kMaxSlots || B > 0x7FFFFFFF) return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if (S <= 1) {  // no score / mask columns: only the error bytes (the kernels write every row's)
    if (!err) return RMI_EINVAL;
    return hipMemsetAsync(err, 0, (size_t)B, as_stream(stream)) == hipSuccess ? RMI_OK : RMI_EDEVICE;
  }
  if (!ids || !n_scores || !score_out || !loss_mask || !response_mask || !err || (T > 0 && !scores))
    return RMI_EINVAL;
  hipLaunchKernelGGL(masks_kernel<false>, dim3((unsigned)B), dim3(64), 0, as_stream(stream), ids, B, S, special_token,
                     reward_token, scores, n_scores, (int)T, (int)n_slots, (int)flags, score_out, loss_mask,
                     response_mask, err, AsmArgs{});
  return launch_status();
}

RMI_API int rmi_assemble_batch(const int64_t* tokens, const int64_t* row_off, int64_t B, int64_t S, int64_t pad_id,
                               int64_t special_token, int64_t reward_token, const double* scores,
                               const int32_t* n_scores, int32_t T, int32_t n_slots, int32_t flags, int64_t* input_ids,
                               int64_t* attention_mask, int64_t* position_ids, float* score_out, uint8_t* loss_mask,
                               uint8_t* response_mask, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || S < 1 || T < 0 || n_slots < 0) return RMI_EINVAL;
  if (n_slots > kMaxSlots || B > 0x7FFFFFFF) return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if (!tokens || !row_off || !input_ids || !attention_mask || !position_ids || !n_scores || !err ||
      (T > 0 && !scores) || (S > 1 && (!score_out || !loss_mask || !response_mask)))
    return RMI_EINVAL;
  hipLaunchKernelGGL(masks_kernel<true>, dim3((unsigned)B), dim3(64), 0, as_stream(stream), nullptr, B, S,
                     special_token, reward_token, scores, n_scores, (int)T, (int)n_slots, (int)flags, score_out,
                     loss_mask, response_mask, err, AsmArgs{tokens, row_off, nullptr, pad_id, input_ids,
                                                            attention_mask, position_ids, nullptr, nullptr});
  return launch_status();
}

RMI_API int rmi_assemble_rows(const int64_t* tokens, const int64_t* row_start, const int32_t* row_len, int64_t B,
                              int64_t S, int64_t pad_id, int64_t special_token, int64_t reward_token,
                              const double* scores, const int32_t* n_scores, int32_t T, int32_t n_slots, int32_t flags,
                              int64_t* input_ids, int64_t* attention_mask, int64_t* position_ids, float* score_out,
                              uint8_t* loss_mask, uint8_t* response_mask, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || S < 1 || T < 0 || n_slots < 0) return RMI_EINVAL;
  if (n_slots > kMaxSlots || B > 0x7FFFFFFF) return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if (!tokens || !row_start || !row_len || !input_ids || !attention_mask || !position_ids || !n_scores || !err ||
      (T > 0 && !scores) || (S > 1 && (!score_out || !loss_mask || !response_mask)))
    return RMI_EINVAL;
  hipLaunchKernelGGL(masks_kernel<true>, dim3((unsigned)B), dim3(64), 0, as_stream(stream), nullptr, B, S,
                     special_token, reward_token, scores, n_scores, (int)T, (int)n_slots, (int)flags, score_out,
                     loss_mask, response_mask, err, AsmArgs{tokens, row_start, row_len, pad_id, input_ids,
                                                            attention_mask, position_ids, nullptr, nullptr});
  return launch_status();
}

RMI_API int rmi_assemble_rows_ex(const int64_t* tokens, const int64_t* row_start, const int32_t* row_len, int64_t B,
                                 int64_t S, int64_t pad_id, int64_t special_token, int64_t reward_token,
                                 const double* scores, const int32_t* n_scores, int32_t T, int32_t n_slots,
                                 int32_t flags, const float* last_score, int64_t* input_ids, int64_t* attention_mask,
                                 int64_t* position_ids, float* score_out, uint8_t* loss_mask, uint8_t* response_mask,
                                 int32_t* resp_count, uint8_t* err, rmi_stream_t stream) {
  using namespace rmi;
  if (B < 0 || S < 1 || T < 0 || n_slots < 0 || (last_score && (flags & RMI_MS_TURN_SCORES))) return RMI_EINVAL;
  if (n_slots > kMaxSlots || B > 0x7FFFFFFF) return RMI_EUNSUP;
  if (B == 0) return RMI_OK;
  if (!tokens || !row_start || !row_len || !input_ids || !attention_mask || !position_ids || !n_scores || !err ||
      (T > 0 && !scores) || (S > 1 && (!score_out || !loss_mask || !response_mask)))
    return RMI_EINVAL;
  if (resp_count && S <= 1)  // no mask columns: no response tokens
    if (hipMemsetAsync(resp_count, 0, (size_t)B * 4, as_stream(stream)) != hipSuccess) return RMI_EDEVICE;
  hipLaunchKernelGGL(masks_kernel<true>, dim3((unsigned)B), dim3(64), 0, as_stream(stream), nullptr, B, S,
                     special_token, reward_token, scores, n_scores, (int)T, (int)n_slots, (int)flags, score_out,
                     loss_mask, response_mask, err,
                     AsmArgs{tokens, row_start, row_len, pad_id, input_ids, attention_mask, position_ids,
                             S > 1 ? resp_count : nullptr, last_score});
  return launch_status();
}
