"""ctypes binding of the C ABI (include/ragen_amd.h) exported by ``_build/libragen_amd.so``.

This is the Python side of the drop-in boundary: the product path always runs the HIP
kernels in this library and fails loudly when the library is missing — there is no CPU
fallback anywhere in ``ragen_amd``.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's libamdhip64 first so the library binds to the same HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
# RAGEN_AMD_LIB: a variant build of the same ABI, for the A/B tools under tools/ only
LIB_PATH = os.environ.get("RAGEN_AMD_LIB") or os.path.join(_HERE, "_build", "libragen_amd.so")

c_int32, c_int64, c_double, c_void_p, c_size_t = (ctypes.c_int32, ctypes.c_int64, ctypes.c_double,
                                                   ctypes.c_void_p, ctypes.c_size_t)

RMI_OK, RMI_EINVAL, RMI_EDEVICE, RMI_EUNSUP = 0, -1, -2, -3
FLAG_TERMINATED, FLAG_TRUNCATED, FLAG_DONE = 1, 2, 4
INFO_PRESENT, INFO_EFFECTIVE, INFO_VALID, INFO_SUCCESS = 1, 2, 4, 8
ERR_ACTION, ERR_INDEX, ERR_STATE, ERR_UNSUP = 1, 2, 4, 8
MS_TURN_SCORES, MS_RESPONSE_MASK, MS_ROLL = 1, 2, 4
BOARDS_NONE, BOARDS_BUILD, BOARDS_USE = 0, 1, 2
NORM_METHODS = {"identity": 0, "mean": 1, "mean_std": 2, "asym_clip": 3}


class Episode(ctypes.Structure):
    _fields_ = [("B", c_int32), ("T", c_int32), ("num_actions", c_void_p), ("flags", c_void_p),
                ("n_turns", c_void_p), ("penalty", c_void_p), ("turn_reward", c_void_p),
                ("turn_info", c_void_p), ("turn_exec", c_void_p)]


class Turn(ctypes.Structure):
    _fields_ = [("turn", c_int32), ("K", c_int32), ("actions", c_void_p), ("n_actions", c_void_p),
                ("has_input", c_void_p), ("max_actions_per_traj", c_int32), ("format_penalty", c_double)]


class Sokoban(ctypes.Structure):
    _fields_ = [("H", c_int32), ("W", c_int32), ("num_boxes", c_int32), ("max_steps", c_int32),
                ("room_fixed", c_void_p), ("room_state", c_void_p), ("player", c_void_p),
                ("num_env_steps", c_void_p), ("boxes_on_target", c_void_p),
                ("boards", c_void_p), ("boards_mode", c_int32), ("init_boards", c_void_p)]


class Finalize(ctypes.Structure):
    _fields_ = [("group_size", c_int32), ("method", c_int32), ("metrics", c_void_p), ("score", c_void_p),
                ("pen", c_void_p), ("norm", c_void_p)]


class Render(ctypes.Structure):
    """rmi_render_t: the observation output of rmi_sokoban_step_turn_render."""
    _fields_ = [("glyph_bytes", ctypes.c_uint32 * 16), ("glyph_len", ctypes.c_uint8 * 16), ("out", c_void_p),
                ("stride", c_int32), ("len", c_void_p)]


class FrozenLake(ctypes.Structure):
    _fields_ = [("nrow", c_int32), ("ncol", c_int32), ("is_slippery", c_int32), ("cs0", c_double),
                ("cs1", c_double), ("cs2", c_double), ("desc", c_void_p), ("s", c_void_p), ("rng", c_void_p)]


class Bandit(ctypes.Structure):
    _fields_ = [("action_space_start", c_int32), ("lo_arm_score", c_double), ("hi_arm_loscore", c_double),
                ("hi_arm_hiscore", c_double), ("hi_arm_hiscore_prob", c_double), ("hi_is_first", c_void_p),
                ("rng", c_void_p)]


class Countdown(ctypes.Structure):
    _fields_ = [("max_nums", c_int32), ("score", c_double), ("format_score", c_double), ("nums", c_void_p),
                ("n_nums", c_void_p), ("target", c_void_p)]


PARSE_MAX_NAMES = 8


class ParseCfg(ctypes.Structure):
    _fields_ = [("enable_think", c_int32), ("prepend", c_int32), ("K", c_int32), ("sep_len", c_int32),
                ("sep_lo", ctypes.c_uint64), ("sep_hi", ctypes.c_uint64), ("n_names", c_int32),
                ("name_len", ctypes.c_uint8 * PARSE_MAX_NAMES), ("name_lo", ctypes.c_uint64 * PARSE_MAX_NAMES),
                ("name_hi", ctypes.c_uint64 * PARSE_MAX_NAMES), ("name_id", (ctypes.c_int8 * PARSE_MAX_NAMES) * 2)]


class TokenRows(ctypes.Structure):
    """rmi_token_rows_t: the decode + parse inputs and outputs of rmi_sokoban_token_turn."""
    _fields_ = [("ids", c_void_p), ("R", c_int64), ("n_ids", c_void_p), ("vocab_packed", c_void_p),
                ("vocab_bytes", c_void_p), ("n_bytes", c_int64), ("V", c_int64), ("text", c_void_p),
                ("stride", c_int32), ("text_len", c_void_p), ("decode_err", c_void_p), ("cfg", ctypes.POINTER(ParseCfg)),
                ("sel", c_void_p), ("spans", c_void_p), ("parse_err", c_void_p), ("has_t", c_void_p),
                ("has", c_void_p)]


PROMPT_MAX_PIECES = 32
PT_CONST, PT_TAG_CONST, PT_OBS, PT_INT, PT_REWARD, PT_RESPONSE, PT_MARK, PT_IF = range(8)


class Piece(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("a", c_int32), ("b", c_int32)]


class Prompt(ctypes.Structure):
    """rmi_prompt_t."""
    _fields_ = [("n_pieces", c_int32), ("pieces", Piece * PROMPT_MAX_PIECES), ("pool", c_void_p),
                ("tag_const", c_void_p), ("n_tags", c_int32), ("tag", c_void_p), ("obs", c_void_p),
                ("obs_stride", c_int32), ("obs_len", c_void_p), ("ints", c_void_p), ("reward", c_void_p),
                ("reward_int", c_void_p), ("resp", c_void_p), ("resp_stride", c_int32), ("resp_len", c_void_p),
                ("spans", c_void_p), ("enable_think", c_int32), ("K", c_int32), ("sep_len", c_int32),
                ("sep", ctypes.c_uint8 * 16), ("cond", c_void_p), ("active", c_void_p),
                ("pool_len", c_int32), ("turn_exec", c_void_p), ("flags", c_void_p),
                ("int_reward_tags", ctypes.c_uint32), ("last_turn", c_int32), ("num_cache", c_void_p),
                ("num_cache_mask", ctypes.c_uint32)]


class TurnChain(ctypes.Structure):
    """rmi_turn_chain_t: one device turn of the rollout loop as one call (rmi_turn_chain)."""
    _fields_ = [("n_envs", c_int64), ("pad_err", c_void_p), ("n_pad", c_int64),
                ("resp", c_void_p), ("n_resp", c_int64), ("R", c_int64), ("src", c_void_p),
                ("vocab_packed", c_void_p), ("vocab_bytes", c_void_p), ("vocab_n_bytes", c_int64), ("V", c_int64),
                ("ids", c_void_p), ("n_ids", c_void_p), ("has_t", c_void_p), ("raw_max", c_void_p),
                ("raw_next", c_void_p),
                ("parse", c_void_p), ("sel", c_void_p), ("text", c_void_p), ("stride", c_int32),
                ("text_len", c_void_p), ("dec_err", c_void_p), ("actions", c_void_p), ("n_actions", c_void_p),
                ("spans", c_void_p), ("parse_err", c_void_p),
                ("has", c_void_p), ("err", c_void_p), ("env_kind", c_int32), ("sokoban", c_void_p),
                ("frozenlake", c_void_p), ("ep", c_void_p), ("turn", c_int32), ("K", c_int32),
                ("max_actions_per_traj", c_int32), ("format_penalty", c_double), ("obs", c_void_p),
                ("max_actions", c_void_p), ("flags_copy", c_void_p), ("left", c_void_p), ("pack", c_void_p),
                ("prompt", c_void_p), ("ptext", c_void_p), ("pstride", c_int32), ("ptext_len", c_void_p),
                ("pmark", c_void_p), ("pterr", c_void_p), ("bpe", c_void_p), ("bpe_stride", c_int32),
                ("arena", c_void_p), ("arena_stride", c_int64), ("arena_len", c_void_p), ("mark_tok", c_void_p),
                ("bpe_err", c_void_p), ("len_upd", c_void_p), ("bad", c_void_p), ("stats", c_void_p),
                ("next_rows", c_void_p), ("next_src", c_void_p),
                ("host", c_void_p), ("pack_bytes", c_int64),
                ("pad_block", c_void_p), ("pad_cap", c_int64), ("pad_tail", c_void_p), ("pad_tail_n", c_int32),
                ("pad_id", c_int64), ("pad_err_next", c_void_p), ("pad_S_out", c_void_p)]


CHAIN_SOKOBAN, CHAIN_FROZENLAKE = 0, 1


class FormulateChain(ctypes.Structure):
    """rmi_formulate_chain_t: formulate_rollouts' update batch as one call (rmi_formulate_chain)."""
    _fields_ = [("ep", c_void_p), ("seg", c_void_p), ("G", c_int32), ("method", c_int32), ("metrics", c_void_p),
                ("norm", c_void_p), ("tokens", c_void_p), ("row_start", c_void_p), ("row_len", c_void_p),
                ("B", c_int64), ("S", c_int64), ("pad_id", c_int64), ("special_token", c_int64),
                ("reward_token", c_int64), ("scores", c_void_p), ("n_scores", c_void_p), ("T", c_int32),
                ("n_slots", c_int32), ("flags", c_int32), ("input_ids", c_void_p), ("attention_mask", c_void_p),
                ("position_ids", c_void_p), ("score_out", c_void_p), ("loss_mask", c_void_p),
                ("response_mask", c_void_p), ("resp_count", c_void_p), ("err", c_void_p), ("tail", c_void_p),
                ("n_copies", c_int32), ("host", c_void_p * 4), ("dev", c_void_p * 4), ("bytes", c_int64 * 4)]

XG_MAX_RANKS = 16
XG_PUBLISH, XG_WAIT = 1, 2
XG_ERR_PEER_BUSY, XG_ERR_ARRIVALS = 1, 2
XG_MEM_UNCACHED, XG_MEM_FINEGRAINED = 0, 1


class XGather(ctypes.Structure):
    """rmi_xgather_t: the one-shot arena exchange of one rank (include/ragen_amd.h)."""
    _fields_ = [("world", c_int32), ("rank", c_int32), ("nbytes", c_int64), ("region", c_void_p * XG_MAX_RANKS),
                ("state", c_void_p), ("err", c_void_p), ("timeout_us", ctypes.c_uint64),
                ("blocks_per_peer", c_int32)]


_P = ctypes.POINTER
_SIGS = {
    "rmi_version": (ctypes.c_char_p, []),
    "rmi_sokoban_step_turn": (c_int32, [_P(Sokoban), _P(Episode), _P(Turn), c_void_p, c_void_p]),
    "rmi_sokoban_step_turn_finalize": (c_int32, [_P(Sokoban), _P(Episode), _P(Turn), c_void_p, _P(Finalize),
                                                 c_void_p]),
    "rmi_sokoban_generate_rooms": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_int32]),
    "rmi_sokoban_generate_rooms_start": (c_void_p, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32,
                                                    c_void_p, c_void_p, c_void_p, c_void_p, c_int32]),
    "rmi_sokoban_generate_rooms_wait": (c_int32, [c_void_p]),
    "rmi_sokoban_reset": (c_int32, [_P(Sokoban), _P(Episode), c_void_p, c_void_p, c_void_p]),
    "rmi_sokoban_load_rooms": (c_int32, [_P(Sokoban), _P(Episode), c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p]),
    "rmi_sokoban_step_turn_first": (c_int32, [_P(Sokoban), _P(Episode), _P(Turn), c_void_p, c_void_p, c_void_p,
                                              c_void_p]),
    "rmi_rollout_finalize": (c_int32, [_P(Episode), c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p]),
    "rmi_frozenlake_step_turn": (c_int32, [_P(FrozenLake), _P(Episode), _P(Turn), c_void_p, c_void_p]),
    "rmi_frozenlake_reset": (c_int32, [_P(FrozenLake), _P(Episode), c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_pcg64_seed": (c_int32, [c_void_p, c_int64, c_int32, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "rmi_frozenlake_step_turn_finalize": (c_int32, [_P(FrozenLake), _P(Episode), _P(Turn), c_void_p, _P(Finalize),
                                                    c_void_p]),
    "rmi_frozenlake_step_turn_first": (c_int32, [_P(FrozenLake), _P(Episode), _P(Turn), c_void_p, c_void_p,
                                                 c_void_p, c_void_p, c_void_p]),
    "rmi_sokoban_step_turn_render": (c_int32, [_P(Sokoban), _P(Episode), _P(Turn), c_void_p, _P(Finalize), c_void_p,
                                               c_void_p, _P(Render), c_void_p]),
    "rmi_sokoban_token_turn": (c_int32, [_P(TokenRows), _P(Sokoban), _P(Episode), _P(Turn), c_void_p, _P(Finalize),
                                         c_void_p, c_void_p, _P(Render), c_void_p]),
    "rmi_sokoban_render": (c_int32, [_P(Sokoban), c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                     c_void_p]),
    "rmi_frozenlake_render": (c_int32, [_P(FrozenLake), c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                        c_void_p]),
    "rmi_bandit_step_turn": (c_int32, [_P(Bandit), _P(Episode), _P(Turn), c_void_p, c_void_p]),
    "rmi_countdown_step_turn": (c_int32, [_P(Countdown), _P(Episode), _P(Turn), c_void_p, c_void_p, c_int32,
                                          c_void_p, c_void_p]),
    "rmi_countdown_reward": (c_int32, [_P(Countdown), c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                       c_void_p, c_void_p]),
    "rmi_rollout_metrics": (c_int32, [_P(Episode), c_void_p, c_void_p]),
    "rmi_trajectory_scores": (c_int32, [_P(Episode), c_void_p, c_void_p, c_void_p]),
    "rmi_group_normalize": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "rmi_filter_groups": (c_int32, [c_void_p, c_int64, c_int32, c_int32, c_double, c_int32, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_row_sum": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "rmi_masks_and_scores": (c_int32, [c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int32,
                                       c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_assemble_batch": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_void_p,
                                     c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_gae": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_double, c_double, c_int32, c_void_p,
                          c_void_p, c_void_p, c_void_p]),
    "rmi_bilevel_gae": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_double, c_double, c_double,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_whiten_scratch_bytes": (c_size_t, [c_int64]),
    "rmi_masked_whiten": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "rmi_whiten_row_stats": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "rmi_masked_whiten_stats": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "rmi_grpo_outcome": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int32, c_double, c_int32,
                                   c_void_p, c_void_p, c_void_p]),
    "rmi_reinforce_pp_returns": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_double, c_void_p, c_void_p,
                                           c_void_p, c_void_p]),
    "rmi_remax": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "rmi_rloo_outcome": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int32, c_void_p, c_void_p,
                                   c_void_p]),
    "rmi_mask_mul": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    "rmi_detokenize": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                 c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "rmi_vocab_pack": (c_int32, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "rmi_detok_parse": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                  c_void_p, c_int32, c_void_p, c_void_p, _P(ParseCfg), c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "rmi_parse_actions": (c_int32, [_P(ParseCfg), c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "rmi_device_copy": (c_int32, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "rmi_stream_synchronize": (c_int32, [c_void_p]),
    "rmi_readback": (c_int32, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "rmi_upload": (c_int32, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "rmi_xgather_region_bytes": (c_int64, [c_int32, c_int64]),
    "rmi_xgather_slot_offset": (c_int64, [c_int32, c_int64, c_int64]),
    "rmi_xgather_blocks_per_peer": (c_int32, [c_int64]),
    "rmi_xgather_alloc": (c_int32, [c_int64, c_int32, _P(c_void_p), c_void_p]),
    "rmi_xgather_open": (c_int32, [c_void_p, _P(c_void_p)]),
    "rmi_xgather_close": (c_int32, [c_void_p]),
    "rmi_xgather_free": (c_int32, [c_void_p]),
    "rmi_xgather": (c_int32, [_P(XGather), c_void_p, c_int32, c_void_p]),
    "rmi_prompt_text": (c_int32, [_P(Prompt), c_int64, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_gen_rows": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p]),
    "rmi_prompt_commit_stats": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_row_counts": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "rmi_gen_rows_chained": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_pad_rows": (c_int32, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_int64, c_int64,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_assemble_rows": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                                    c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_bpe_encode": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_void_p, c_int64,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_turn_inputs": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "rmi_turn_readback": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                    c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_prompt_commit": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "rmi_rows_stats": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "rmi_next_rows_stats": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "rmi_turn_chain": (c_int32, [_P(TurnChain), c_void_p]),
    "rmi_host_live_ids": (ctypes.c_int64, [c_void_p, c_int64, ctypes.c_uint32, c_int64, c_void_p, c_int64]),
    "rmi_turn_readback_pad": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "rmi_next_rows_list": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "rmi_formulate_stats": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "rmi_formulate_tail": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "rmi_assemble_rows_ex": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                                       c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rmi_formulate_chain": (c_int32, [_P(FormulateChain), c_void_p]),
    "rmi_formulate_chain_part": (c_int32, [_P(FormulateChain), c_int32, c_int32, c_void_p]),
    "rmi_formulate_chain_wait": (c_int32, [c_void_p]),
}

_lib = None


def lib():
    """Load the library (once).  Raises if it has not been built — no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"ragen_amd native library missing: {LIB_PATH}. Build it with `python -m ragen_amd.build` "
                              "(hipcc, gfx950). The engine has no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(rc, what):
    if rc == RMI_OK:
        return
    if rc == RMI_EINVAL:
        raise ValueError(f"{what}: invalid argument (RMI_EINVAL)")
    if rc == RMI_EUNSUP:
        raise NotImplementedError(f"{what}: configuration outside the kernel envelope (RMI_EUNSUP)")
    raise RuntimeError(f"{what}: HIP launch failed (code {rc})")
