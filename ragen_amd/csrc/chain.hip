// chain.cpp — rmi_turn_chain: one device turn of the rollout loop as one host call (host code:
// it only sequences the library's own entry points on the caller's stream; include/ragen_amd.h).
//
// The Python turn loop paid ~20-60 us of interpreter and dispatcher work per launch between the
// turn's ~10 launches (profiles/r04_api_host_stamps.txt: ~400 us of host time per 8192-env turn
// against ~290 us of kernels), so the GPU idled between them.  Enqueued from here the launches
// go back to back and the host's share of a turn is this call plus the Python that reads its
// readback.
#include "common.hpp"

namespace {

// one event per (host thread, device), created on first use: the readback is waited on through
// it, so work enqueued after the copy (the next batch's row list) runs while the host reads the
// copy.  Per thread: two threads running chains on one device must not wait on each other's
// record (each would read its readback tail before its own copy had landed).
hipEvent_t copy_event() {
  thread_local hipEvent_t ev[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!ev[dev] && hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming) != hipSuccess) ev[dev] = nullptr;
  return ev[dev];
}

}  // namespace

RMI_API int rmi_turn_chain(const rmi_turn_chain_t* chain, rmi_stream_t s) {
  if (!chain) return RMI_EINVAL;
  const rmi_turn_chain_t& c = *chain;
  const int64_t B = c.n_envs;
  if (B < 1 || !c.ep || c.ep->B != B || !c.obs || !c.pack || !c.host || c.pack_bytes < 1 || !c.parse ||
      (c.env_kind == RMI_CHAIN_SOKOBAN ? !c.sokoban : c.env_kind == RMI_CHAIN_FROZENLAKE ? !c.frozenlake : true))
    return RMI_EINVAL;
  // the next batch's row list and its pad read the readback tail's stats (longest, any_bad,
  // count), which only step 6's rmi_prompt_commit_stats writes: without a prompt they are stale
  if ((c.next_rows || c.pad_block) && (!c.prompt || !c.stats)) return RMI_EINVAL;
  int rc;
  // 1. the generations onto the env rows (the longest one's raw bytes into the readback)
  if (c.resp) {
    rc = rmi_gen_rows_chained(c.resp, c.n_resp, c.R, c.src, B, c.vocab_packed, c.V, c.src ? c.ids : nullptr,
                              c.src ? c.n_ids : nullptr, c.src ? c.has_t : nullptr, c.raw_max, c.raw_next, s);
    if (rc) return rc;
  }
  // 2-4. decode + parse; the envs that step (a generation, decoded without error; the step errors
  //      zeroed); the turn and the next observation.  Sokoban: one launch (rmi_sokoban_token_turn,
  //      which runs the three steps' launches itself for layouts it does not fuse)
  rmi_turn_t in;
  in.turn = c.turn;
  in.K = c.K;
  in.actions = c.actions;
  in.n_actions = c.n_actions;
  in.has_input = c.has;
  in.max_actions_per_traj = c.max_actions_per_traj;
  in.format_penalty = c.format_penalty;
  if (c.env_kind == RMI_CHAIN_SOKOBAN) {
    rmi_token_rows_t tok;
    tok.ids = c.ids;
    tok.R = c.R;
    tok.n_ids = c.n_ids;
    tok.vocab_packed = c.vocab_packed;
    tok.vocab_bytes = c.vocab_bytes;
    tok.n_bytes = c.vocab_n_bytes;
    tok.V = c.V;
    tok.text = c.text;
    tok.stride = c.stride;
    tok.text_len = c.text_len;
    tok.decode_err = c.dec_err;
    tok.cfg = c.parse;
    tok.sel = c.sel;
    tok.spans = c.spans;
    tok.parse_err = c.parse_err;
    tok.has_t = c.has_t;
    tok.has = c.has;
    rc = rmi_sokoban_token_turn(&tok, c.sokoban, c.ep, &in, c.err, nullptr, nullptr, nullptr, c.obs, s);
  } else {
    rc = rmi_detok_parse(c.ids, B, c.R, c.n_ids, c.vocab_packed, c.vocab_bytes, c.vocab_n_bytes, c.V, c.text,
                         c.stride, c.text_len, c.dec_err, c.parse, c.sel, c.actions, c.n_actions, c.spans, nullptr,
                         nullptr, 0, c.parse_err, s);
    if (!rc) rc = rmi_turn_inputs(c.has_t, c.dec_err, B, c.has, c.err, s);
    if (!rc) rc = rmi_frozenlake_step_turn(c.frozenlake, c.ep, &in, c.err, s);
    if (!rc)
      rc = rmi_frozenlake_render(c.frozenlake, (int32_t)B, c.obs->glyph_bytes, c.obs->glyph_len, c.obs->out,
                                 c.obs->stride, c.obs->len, s);
  }
  if (rc) return rc;
  // 5. the record's flags / actions-left columns and the packed readback (the batch's left-cut rows counted)
  rc = rmi_turn_readback_pad(c.ep->flags, c.err, c.dec_err, c.ep->num_actions, c.max_actions, c.text_len,
                             c.obs->len, B, c.flags_copy, c.left, c.pack, c.pad_err, c.n_pad, s);
  if (rc) return rc;
  // 6. the next prompt's text, its ids appended to the arena, the commit and the next batch's stats
  if (c.prompt) {
    rc = rmi_prompt_text(c.prompt, B, c.ptext, c.pstride, c.ptext_len, c.pmark, c.pterr, s);
    if (rc) return rc;
    rc = rmi_bpe_encode(c.bpe, c.ptext, c.pstride, c.bpe_stride, c.ptext_len, B, c.arena, c.arena_stride,
                        c.arena_len, nullptr, c.pmark, c.mark_tok, c.bpe_err, s);
    if (rc) return rc;
    rc = rmi_prompt_commit_stats(c.bpe_err, c.pterr, c.has, c.mark_tok, c.len_upd, B, c.bad, c.arena_len, c.has,
                                 c.flags_copy, c.stats, s);
    if (rc) return rc;
  }
  // 7-8. the one readback of the turn, then the next generation batch's rows (enqueued behind the
  // copy and run while the host reads it: the host waits for the copy alone)
  if (!c.next_rows) return rmi_readback(c.host, c.pack, (size_t)c.pack_bytes, s);
  hipStream_t hs = rmi::as_stream(s);
  hipEvent_t ev = copy_event();
  if (!ev) return RMI_EDEVICE;
  rc = rmi::readback_async(c.host, c.pack, (size_t)c.pack_bytes, hs);
  if (rc) return rc;
  if (hipEventRecord(ev, hs) != hipSuccess) return RMI_EDEVICE;
  rc = rmi_next_rows_list(c.has, c.flags_copy, B, c.next_rows, c.next_src, s);
  if (rc) return rc;
  if (hipEventSynchronize(ev) != hipSuccess) return RMI_EDEVICE;
  // 8. the next generation batch, padded while the host reads the readback (its width is in it)
  if (!c.pad_block) return RMI_OK;
  if (!c.pad_S_out) return RMI_EINVAL;
  *c.pad_S_out = 0;
  const int64_t off = (3 * B + 3) & ~(int64_t)3;
  if (c.pack_bytes < off + 20) return RMI_EINVAL;
  const int32_t* tail = reinterpret_cast<const int32_t*>(static_cast<const uint8_t*>(c.host) + off);
  const int64_t longest = tail[2], any_bad = tail[3], count = tail[4];
  if (any_bad || count < 1 || count > B || longest < 0) return RMI_OK;
  const int64_t S = longest + c.pad_tail_n;
  const int64_t P = (count * S + 1) & ~(int64_t)1;  // the outputs at k * P: 16-B aligned alike (column pairs)
  if (S < 1 || 3 * P > c.pad_cap) return RMI_OK;
  rc = rmi_pad_rows(c.arena, c.arena_stride, c.arena_len, c.next_rows, count, c.pad_tail, c.pad_tail_n, S, c.pad_id,
                    c.pad_block, c.pad_block + P, c.pad_block + 2 * P, c.pad_err_next, s);
  if (rc) return rc;
  *c.pad_S_out = S;
  return RMI_OK;
}

namespace {

// the chain's launches and copies, whole (part 0) or in two parts: part 1 = step 1 (the finalize)
// and copies [0, n_early), part 2 = steps 2-3 (the assembly, the tail) and copies [n_early,
// n_copies).  Nothing is waited on here.
int formulate_enqueue(const rmi_formulate_chain_t* chain, int part, int n_early, rmi_stream_t s) {
  if (!chain) return RMI_EINVAL;
  const rmi_formulate_chain_t& c = *chain;
  if (!c.ep || c.ep->B != c.B || !c.norm || !c.tail || c.n_copies < 0 || c.n_copies > 4 ||
      (c.flags & RMI_MS_TURN_SCORES) || part < 0 || part > 2 || n_early < 0 || n_early > c.n_copies)
    return RMI_EINVAL;
  hipStream_t hs = rmi::as_stream(s);
  int rc;
  if (part != 2) {
    rc = rmi_rollout_finalize(c.ep, c.seg, c.G, c.method, c.metrics, nullptr, nullptr, c.norm, s);
    if (rc) return rc;
    for (int i = 0; i < n_early; ++i)
      if (c.bytes[i] > 0 && (rc = rmi::readback_async(c.host[i], c.dev[i], (size_t)c.bytes[i], hs)) != RMI_OK)
        return rc;
    if (part == 1) return RMI_OK;
  }
  rc = rmi_assemble_rows_ex(c.tokens, c.row_start, c.row_len, c.B, c.S, c.pad_id, c.special_token, c.reward_token,
                            c.scores, c.n_scores, c.T, c.n_slots, c.flags, c.norm, c.input_ids, c.attention_mask,
                            c.position_ids, c.score_out, c.loss_mask, c.response_mask, c.resp_count, c.err, s);
  if (rc) return rc;
  rc = rmi_formulate_tail(c.resp_count, c.err, c.B, c.tail, s);
  if (rc) return rc;
  for (int i = n_early; i < c.n_copies; ++i)
    if (c.bytes[i] > 0 && (rc = rmi::readback_async(c.host[i], c.dev[i], (size_t)c.bytes[i], hs)) != RMI_OK) return rc;
  return RMI_OK;
}

}  // namespace

RMI_API int rmi_formulate_chain(const rmi_formulate_chain_t* chain, rmi_stream_t s) {
  const int rc = formulate_enqueue(chain, 0, 0, s);
  if (rc) return rc;
  return hipStreamSynchronize(rmi::as_stream(s)) == hipSuccess ? RMI_OK : RMI_EDEVICE;
}

RMI_API int rmi_formulate_chain_part(const rmi_formulate_chain_t* chain, int32_t part, int32_t n_early,
                                     rmi_stream_t s) {
  if (part != 1 && part != 2) return RMI_EINVAL;
  return formulate_enqueue(chain, part, n_early, s);
}

RMI_API int rmi_formulate_chain_wait(rmi_stream_t s) {
  return hipStreamSynchronize(rmi::as_stream(s)) == hipSuccess ? RMI_OK : RMI_EDEVICE;
}
