"""Benchmark: env-steps/sec of the batched Sokoban rollout (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N      (one rank per GPU)

Workload (BASELINE.json configs[2], SURVEY §8(d) "SK"): Sokoban 6x6 / 1 box, 8192 envs per
GPU (512 groups x 16, env i seeded 1000 + i // 16), 5 turns of up to K=5 synthetic actions
per env (10 % unknown names), max 10 actions per trajectory.  One bench "step" = one whole
rollout phase over the batch from the post-reset state (room generation is excluded, as
§8(d) specifies; the device restore of the reset state is fused into the first turn), 5 turn
kernels, get_rollout_states metrics, trajectory scores and the StarPO reward normalisation
(fused into the last turn).  Inputs are resident in HBM before timing.  The step is captured
in a HIP graph and replayed, several rollouts per replay.

Multi-GPU: weak scaling — every rank runs its own 8192 envs (global group ids preserved,
rank r seeds groups r*512..), no collective on the data path; value = all ranks' env steps
/ max-over-ranks time.

Also reported: roofline of the dominant kernel (rmi_sokoban_step_turn) — algorithmic bytes
(141 B per active env-turn) over the average launch duration measured with HIP
events around back-to-back launches — PMC HBM traffic per launch from the committed
rocprofv3 pass (profiles/), and the CPU baseline (the oracle's per-env Python port of the
reference path, timed on this host).
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as tdist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from ragen_amd import distributed as rd  # noqa: E402
from ragen_amd import _lib, ops, synthetic  # noqa: E402
from ragen_amd.env import SokobanBatch  # noqa: E402
from ragen_amd.env.configs import SokobanEnvConfig  # noqa: E402

B_PER_GPU = 8192
T_TURNS = 5
K_ACTIONS = 5
MAX_ACTIONS = 10
GROUP = 16
BYTES_PER_ENV_TURN = 141  # algorithmic bytes per Sokoban env-turn
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured copy)
ROLLOUTS_PER_GRAPH = 8    # extras legs: rollouts per graph replay (the headline's --group default)
PMC_GLOB = os.path.join(ROOT, "profiles", "r*_pmc_sokoban_step_turn.json")  # latest round's PMC pass
PMC_SCALE_GLOB = os.path.join(ROOT, "profiles", "r*_pmc_sokoban_4M.json")  # the at-scale leg's PMC pass


def _pmc_field(pattern, key):
    """A field of the newest committed PMC summary (profiles/rNN_*.json), or None."""
    files = sorted(glob.glob(pattern))
    if not files:
        return None
    with open(files[-1]) as f:
        return json.load(f).get(key)


def _pmc_source(pattern):
    """Where the line's PMC traffic figures come from (a counter pass cannot run inside the timed
    process): the newest committed summary and the counter runs it was computed from."""
    files = sorted(glob.glob(pattern))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    return {"file": os.path.relpath(files[-1], ROOT), "from": d.get("source"), "workload": d.get("workload")}


ISSUE_GLOB = os.path.join(ROOT, "profiles", "r*_issue_frac.json")  # the text kernels' issue-rate pass


def attach_issue_fracs(text):
    """The text kernels are bound by instruction issue, not HBM (their `frac` of 8 TB/s is near
    zero): each text_api block gets the issue-rate figures of the newest committed PMC pass
    (tools/r06_issue_pmc.sh, tools/issue_frac.py) -- instructions per launch and durations from
    the same profiled launches (a counter pass cannot run inside the timed process)."""
    files = sorted(glob.glob(ISSUE_GLOB))
    if not files:
        return
    with open(files[-1]) as f:
        d = json.load(f)
    where = {"parse": ("parse",), "detok": ("detokenize",), "detok_parse": ("detok_parse",),
             "token_turn": ("token_rollout",), "bpe_encode": ("prompt", "bpe_encode"),
             "prompt_text": ("prompt", "prompt_text")}
    for k, path in where.items():
        v = d["kernels"].get(k)
        blk = text
        for p in path:
            blk = blk.get(p) if isinstance(blk, dict) else None
        if v is None or not isinstance(blk, dict):
            continue
        blk["issue_frac"] = v["issue_frac"]
        blk["valu_frac"] = v["valu_frac"]
        blk["salu_frac"] = v["salu_frac"]
        blk["issue_source"] = {"file": os.path.relpath(files[-1], ROOT), "profiled_avg_us": v["avg_us"],
                               "insts_per_wave": v["per_wave"], "definition": d["definition"]}


class Rollout:
    """The SK rollout on one rank.  boards: the turn launches keep the board cache
    (SokobanBatch.enable_boards): the first turn of a rollout builds it (a fresh episode always
    does), the later turns read one 16-B entry per env instead of the two grid rows and skip
    their decode."""

    def __init__(self, device, rank, B=B_PER_GPU, boards=True):
        self.device = device
        self.B = B
        cfg = SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100)
        self.env = SokobanBatch(cfg, B, T_TURNS, K_ACTIONS, device)
        first_group = rank * (B // GROUP)
        self.env.reset(synthetic.env_seeds(B, synthetic.ENV_SEED, GROUP, first_group))
        e = self.env
        ids, n = synthetic.rollout_actions(B, T_TURNS, K_ACTIONS, 1, 4, seed=synthetic.ACTION_SEED + rank)
        self.ids = torch.from_numpy(ids).to(device)
        self.n = torch.from_numpy(n).to(device)
        self.seg = torch.arange(0, B + 1, GROUP, dtype=torch.int32, device=device)
        self.norm = torch.empty(B, dtype=torch.float32, device=device)
        self.metrics = torch.empty(B, 4, dtype=torch.float64, device=device)
        self.turns = [ops.turn_struct(t, self.ids[t], self.n[t], None, MAX_ACTIONS, -0.1) for t in range(T_TURNS)]
        self.st = e.struct()
        self.boards = bool(boards) and e.enable_boards()
        # turn 0 (after a restore or fused with it) builds the cache, turns 1.. use it; the fused
        # first turn builds the reset state's entries once, and later rollouts' first turns read them
        self.st_first = e.board_struct(_lib.BOARDS_BUILD) if self.boards else self.st
        self.st_first_use = e.board_struct(_lib.BOARDS_USE) if self.boards else self.st
        self.st_next = e.board_struct(_lib.BOARDS_USE) if self.boards else self.st
        self.fin = ops.finalize_struct(GROUP, "identity", self.norm, self.metrics)

    def step(self):
        """One rollout phase from the post-reset state: T turn launches.  The first is fused with
        the reset's restore (rmi_sokoban_step_turn_first == rmi_sokoban_reset + turn, tested bit
        for bit), the last with the rollout's finalize (metrics + scores + normalisation ==
        rmi_rollout_finalize, tested bit for bit)."""
        e = self.env
        first = self.st_first_use if e.init_boards_valid else self.st_first
        ops.sokoban_step_turn_first(first, e.ep, self.turns[0], e.init_state, e.init_player)
        e.init_boards_valid = self.boards
        for t in range(1, T_TURNS - 1):
            ops.sokoban_step_turn(self.st_next, e.ep, self.turns[t])
        ops.sokoban_step_turn_finalize(self.st_next, e.ep, self.turns[-1], self.fin)

    def step_unfused(self):
        """The same rollout with T plain turn launches and the separate finalize launch (the
        dominant kernel alone, for the roofline and PMC passes)."""
        self.env.restore()
        for t in range(T_TURNS):
            ops.sokoban_step_turn(self.st_next if t else self.st_first, self.env.ep, self.turns[t])
        ops.rollout_finalize(self.env.ep, self.seg, "identity", self.norm, metrics=self.metrics)

    def timed_turns(self):
        """One rollout phase with HIP events (on the launch stream) around its T back-to-back
        turn launches.  A spin kernel queued first keeps the GPU busy while the host enqueues,
        so no host gap falls inside the bracket.  -> (start, end) events."""
        torch.cuda._sleep(2_000_000)
        self.env.restore()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for t in range(T_TURNS):
            ops.sokoban_step_turn(self.st_next if t else self.st_first, self.env.ep, self.turns[t])
        b.record()
        ops.rollout_finalize(self.env.ep, self.seg, "identity", self.norm, metrics=self.metrics)
        return a, b


def scale_leg(R, device, tile=512, reps=5):
    """The dominant kernel where HBM, not launch latency, bounds it: the bench's 8192 envs
    tiled `tile` times (4 194 304 envs: ~484 MB of algorithmic traffic per launch and a ~420 MB
    footprint, past the 256 MiB Infinity Cache, so every launch streams from HBM), 5 turns,
    HIP events around the turn launches.  Same rooms and actions in every tile, so each
    turn's active count is exactly tile x the bench's.  -> (seconds per 5 launches, envs)."""
    B = R.B * tile
    env = SokobanBatch(SokobanEnvConfig(dim_x=6, dim_y=6, num_boxes=1, max_steps=100), B, T_TURNS, K_ACTIONS, device)
    env.room_fixed.copy_(R.env.room_fixed.repeat(tile, 1))
    env.init_state.copy_(R.env.init_state.repeat(tile, 1))
    env.init_player.copy_(R.env.init_player.repeat(tile, 1))
    ids = R.ids.repeat(1, tile, 1).contiguous()
    n = R.n.repeat(1, tile).contiguous()
    turns = [ops.turn_struct(t, ids[t], n[t], None, MAX_ACTIONS, -0.1) for t in range(T_TURNS)]
    st = env.struct()
    ev = []
    for r in range(reps + 1):
        env.restore()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for t in range(T_TURNS):
            ops.sokoban_step_turn(st, env.ep, turns[t])
        b.record()
        if r:
            ev.append((a, b))
    torch.cuda.synchronize()
    steps = int(env.ep.turn_exec.sum().item())
    assert steps == tile * int(R.env.ep.turn_exec.sum().item()), "tiled rollout diverged from the bench's"
    dur = float(np.mean([x.elapsed_time(y) for x, y in ev])) * 1e-3
    del env, ids, n
    return dur, B


def layout_floor(active, hw=36, all_env_bytes=(1, 2, 1, 1, 1, 1, 8, 1, 5), lines=(64, 128)):
    """The least HBM read traffic per launch that the turn kernel's access contract allows, for
    the scale leg's plain turns: the caller-owned SoA keeps done envs
    interleaved with acting ones, so every env's lane reads its flags and scalars (flags,
    player, num_env_steps, boxes_on_target, num_actions, n_turns, penalty, n_actions, actions:
    21 B) and the two grids (room_state, room_fixed) are read wherever an acting env's row
    touches a line.  active: bool[T, B] per turn.  -> {line: MB per launch (mean over turns)}."""
    T, B = active.shape
    out = {}
    for line in lines:
        full = sum(-(-B * sz // line) * line for sz in all_env_bytes)
        tot = 0
        for t in range(T):
            idx = np.nonzero(active[t])[0].astype(np.int64)
            touched = np.zeros(-(-B * hw // line), bool)
            touched[(idx * hw) // line] = True
            touched[(idx * hw + hw - 1) // line] = True
            tot += full + 2 * int(touched.sum()) * line
        out[line] = tot / T / 1e6
    return out


GUIDE_COPY_GBS = 6290.0  # MI355X_MICROARCH.md: HBM3E 6.29 TB/s measured (float4 copy)


def hbm_copy_peak(device, nbytes=1 << 30, reps=10):
    """Achievable HBM bandwidth on this box: rmi_device_copy (the library's 16-B-per-lane
    grid-stride streaming copy, MI355X_MICROARCH.md's float4-copy recipe) of 1 GiB, read +
    write, far past the 256 MiB Infinity Cache; HIP events on the launch stream."""
    from ragen_amd._lib import check, lib
    x = torch.empty(nbytes, dtype=torch.uint8, device=device)
    y = torch.empty_like(x)
    s = torch.cuda.current_stream(device)

    def copy():
        check(lib().rmi_device_copy(y.data_ptr(), x.data_ptr(), nbytes, s.cuda_stream), "rmi_device_copy")
    copy()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        copy()
    b.record(s)
    torch.cuda.synchronize()
    gbs = 2 * nbytes * reps / (a.elapsed_time(b) * 1e-3) / 1e9
    del x, y
    return gbs


def advantage_leg(R, device, reps=20):
    """The StarPO advantage step on this rollout's trajectories (compute_advantage hot path):
    token rows [B, L] in SURVEY §8(d)'s synthetic layout (150-token prompt, per executed turn a
    state block + a response block, score at the last column), verl GAE (legacy, gamma = lam = 1)
    with fp64 per-row whitening partials, then masked whitening.  Timed with HIP events around
    back-to-back launches; algorithmic bytes 17 per token (r, V, mask in; adv, ret out)."""
    n_turns = R.env.ep.n_turns.cpu().numpy()
    score = R.norm.cpu().numpy()
    r, v, m = synthetic.token_rows(n_turns, score, seed=11)
    r, v, m = (torch.from_numpy(x).to(device) for x in (r, v, m))
    B, L = r.shape
    stats = torch.empty(B, 3, dtype=torch.float64, device=device)
    for _ in range(3):
        adv, ret = ops.gae(r, v, m, 1.0, 1.0, row_stats=stats)
        ops.masked_whiten_(adv, m, stats)
    torch.cuda._sleep(2_000_000)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    for _ in range(reps):
        adv, ret = ops.gae(r, v, m, 1.0, 1.0, row_stats=stats)
    e[1].record()
    for _ in range(reps):
        ops.masked_whiten_(adv, m, stats)
    e[2].record()
    torch.cuda.synchronize()
    gae_us = e[0].elapsed_time(e[1]) * 1e3 / reps
    whiten_us = e[1].elapsed_time(e[2]) * 1e3 / reps
    tokens = B * L
    gbs = tokens * 17 / (gae_us * 1e-6) / 1e9
    del adv, ret
    # the same estimator past the 256 MiB Infinity Cache: the rows left-padded to 4096 tokens
    # (8192 x 4096 = 33.5 M tokens, 570 MB of algorithmic traffic per launch)
    r4, v4, m4 = (torch.from_numpy(x).to(device) for x in synthetic.token_rows(n_turns, score, seed=11, max_len=4096))
    s4 = torch.empty(B, 3, dtype=torch.float64, device=device)
    a4, t4 = ops.gae(r4, v4, m4, 1.0, 1.0, row_stats=s4)
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(5):
        a4, t4 = ops.gae(r4, v4, m4, 1.0, 1.0, row_stats=s4)
    e[1].record()
    for _ in range(5):
        ops.masked_whiten_(a4, m4, s4)
    e[2].record()
    torch.cuda.synchronize()
    tok4 = r4.numel()
    gae4_us = e[0].elapsed_time(e[1]) * 1e3 / 5
    whiten4_us = e[1].elapsed_time(e[2]) * 1e3 / 5
    out_of_cache = {"rows": B, "cols": r4.shape[1], "tokens_per_launch": tok4, "gae_us": gae4_us,
                    "achieved_GBs": tok4 * 17 / (gae4_us * 1e-6) / 1e9,
                    "frac": tok4 * 17 / (gae4_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                    "whiten_us": whiten4_us, "whiten_GBs": tok4 * 8 / (whiten4_us * 1e-6) / 1e9,
                    "cache": "out of the 256 MiB Infinity Cache (570 MB per GAE launch)",
                    "traffic": _pmc_field(os.path.join(ROOT, "profiles", "r*_pmc_gae_4096.json"),
                                          "hbm_bytes_per_launch")}
    del r4, v4, m4, a4, t4, s4
    # get_masks_and_scores (rmi_masks_and_scores) on token ids of the same [B, L+1] shape:
    # 8 B/token in (ids), 6 B/token out (score f32 + two masks)
    g = torch.Generator(device=device).manual_seed(3)
    ids = torch.randint(100, 1000, (B, L + 1), generator=g, device=device, dtype=torch.int64)
    ids[torch.rand(B, L + 1, generator=g, device=device) < 0.02] = 151644
    ids[torch.rand(B, L + 1, generator=g, device=device) < 0.01] = 151645
    n_sc = R.env.ep.n_turns.to(torch.int32)
    for _ in range(3):
        ops.masks_and_scores(ids, 151644, 151645, R.env.ep.turn_reward, n_sc, T_TURNS, False, True, True)
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        ops.masks_and_scores(ids, 151644, 151645, R.env.ep.turn_reward, n_sc, T_TURNS, False, True, True)
    e[1].record()
    torch.cuda.synchronize()
    masks_us = e[0].elapsed_time(e[1]) * 1e3 / reps
    mgbs = B * (L + 1) * 14 / (masks_us * 1e-6) / 1e9
    # the whole formulate batch in one pass (rmi_assemble_batch): ragged rows (the same ids, each
    # row cut to its own length) -> padded ids, attention_mask, position_ids, masks, scores;
    # 8 B/token in, 30 B/token out (3 x i64, f32 score, 2 masks)
    lens = torch.randint(L // 2, L + 2, (B,), generator=g, device=device)
    keep = torch.arange(L + 1, device=device)[None, :] < lens[:, None]
    toks = ids[keep].contiguous()
    off = torch.zeros(B + 1, dtype=torch.int64, device=device)
    off[1:] = torch.cumsum(lens, 0)
    S_asm = int(lens.max())
    for _ in range(3):
        ops.assemble_batch(toks, off, S_asm, 151643, 151644, 151645, R.env.ep.turn_reward, n_sc, T_TURNS, False,
                           True, True)
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        ops.assemble_batch(toks, off, S_asm, 151643, 151644, 151645, R.env.ep.turn_reward, n_sc, T_TURNS, False,
                           True, True)
    e[1].record()
    torch.cuda.synchronize()
    asm_us = e[0].elapsed_time(e[1]) * 1e3 / reps
    asm_bytes = toks.numel() * 8 + B * S_asm * 24 + B * (S_asm - 1) * 6
    assemble = {"kernel": "rmi_assemble_batch", "rows": B, "S": S_asm, "tokens": int(toks.numel()), "us": asm_us,
                "achieved_GBs": asm_bytes / (asm_us * 1e-6) / 1e9, "frac": asm_bytes / (asm_us * 1e-6) / 1e9 /
                HBM_PEAK_GBS, "bytes": int(asm_bytes)}
    del toks, keep
    # bi-level GAE (turn-level rewards at each turn's last response token) and GRPO outcome
    tr = R.env.ep.turn_reward.t().contiguous().cpu().numpy().astype(np.float32)
    tr[tr == 0] = 0.5  # a zero turn reward would end the row's high-level segment early
    rb, vb, mb = synthetic.token_rows(n_turns, score, seed=12, turn_scores=tr)
    rb, vb, mb = (torch.from_numpy(x).to(device) for x in (rb, vb, mb))
    seg = torch.arange(0, rb.shape[0] + 1, dtype=torch.int32, device=device)
    for _ in range(2):
        ops.bilevel_gae(rb, vb, mb, 1.0, 0.95, 0.95, check_errors=False)
        ops.grpo_outcome(rb, mb, seg)
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        ops.bilevel_gae(rb, vb, mb, 1.0, 0.95, 0.95, check_errors=False)
    e[1].record()
    for _ in range(reps):
        ops.grpo_outcome(rb, mb, seg)
    e[2].record()
    torch.cuda.synchronize()
    bl_us = e[0].elapsed_time(e[1]) * 1e3 / reps
    grpo_us = e[1].elapsed_time(e[2]) * 1e3 / reps
    tok_b = rb.shape[0] * rb.shape[1]
    del rb, vb, mb
    # bi-level GAE past the Infinity Cache: the same turn-score rows left-padded to 4096 tokens
    # (8192 x 4096: 570 MB of algorithmic traffic per launch), as GAE's out_of_cache
    rb4, vb4, mb4 = (torch.from_numpy(x).to(device)
                     for x in synthetic.token_rows(n_turns, score, seed=12, turn_scores=tr, max_len=4096))
    ops.bilevel_gae(rb4, vb4, mb4, 1.0, 0.95, 0.95, check_errors=False)
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(5):
        ops.bilevel_gae(rb4, vb4, mb4, 1.0, 0.95, 0.95, check_errors=False)
    e[1].record()
    torch.cuda.synchronize()
    bl4_us = e[0].elapsed_time(e[1]) * 1e3 / 5
    tok_b4 = rb4.numel()
    bl_out = {"rows": rb4.shape[0], "cols": rb4.shape[1], "tokens_per_launch": tok_b4, "us": bl4_us,
              "achieved_GBs": tok_b4 * 17 / (bl4_us * 1e-6) / 1e9,
              "frac": tok_b4 * 17 / (bl4_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
              "cache": "out of the 256 MiB Infinity Cache (570 MB per launch)",
              "traffic": _pmc_field(os.path.join(ROOT, "profiles", "r*_pmc_bilevel_4096.json"), "hbm_bytes_per_launch")}
    del rb4, vb4, mb4
    return {"kernel": "rmi_gae (legacy) + row stats", "rows": B, "cols": L, "tokens_per_launch": tokens,
            "cache": "in the Infinity Cache (152 MB per launch, repeated on the same buffers)",
            "out_of_cache": out_of_cache,
            "gae_us": gae_us, "whiten_us": whiten_us, "tokens_per_s": tokens / ((gae_us + whiten_us) * 1e-6),
            "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS, "bytes_per_token": 17,
            "masks_and_scores": {"kernel": "rmi_masks_and_scores", "us": masks_us, "achieved_GBs": mgbs,
                                 "frac": mgbs / HBM_PEAK_GBS, "bytes_per_token": 14},
            "assemble_batch": assemble,
            "bilevel_gae": {"kernel": "rmi_bilevel_gae", "tokens": tok_b, "us": bl_us,
                            "achieved_GBs": tok_b * 17 / (bl_us * 1e-6) / 1e9, "out_of_cache": bl_out},
            "grpo": {"kernel": "rmi_grpo_outcome", "tokens": tok_b, "us": grpo_us,
                     "achieved_GBs": tok_b * 13 / (grpo_us * 1e-6) / 1e9}}


def _graph_rollout(step, reps=50, warmup=5, per_graph=ROLLOUTS_PER_GRAPH):
    """Capture per_graph back-to-back rollouts (step() each, every one starting from the reset
    state) in one HIP graph, as the headline does, replay it, -> ms per rollout.  The ~7 us
    boundary between graph replays is paid once per per_graph rollouts."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            step()
    for _ in range(warmup):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * per_graph) * 1e3


def toytext_legs(device):
    """BASELINE configs[1] and [4] on this GPU (parity cases of the bench, reported as extras):
    FrozenLake 4x4 slippery, 4096 envs x 8 turns (K=5, cap 10), and Countdown 16384 envs x 4
    turns (K=1, cap 1; half the turns carry no answer -> mixed episode lengths).  Each also
    reports its algorithmic bytes (SURVEY §8(d) per env-turn) over the whole rollout's time.  A rollout =
    T turn launches from the post-reset state (FrozenLake's first one fused with the device
    restore; Countdown's record zeroed), then the fused finalize."""
    from ragen_amd.env import CountdownBatch, FrozenLakeBatch
    from ragen_amd.env.configs import CountdownEnvConfig, FrozenLakeEnvConfig
    from ragen_amd.env.countdown import synthetic_instances
    out = {}
    # FrozenLake
    B, T, K = 4096, 8, 5
    fl = FrozenLakeBatch(FrozenLakeEnvConfig(), B, T, K, device)
    fl.reset(synthetic.env_seeds(B))
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4, seed=synthetic.ACTION_SEED + 1)
    ids, n = torch.from_numpy(ids).to(device), torch.from_numpy(n).to(device)
    seg = torch.arange(0, B + 1, GROUP, dtype=torch.int32, device=device)
    norm = torch.empty(B, dtype=torch.float32, device=device)
    turns = [ops.turn_struct(t, ids[t], n[t], None, 10, -0.1) for t in range(T)]
    st = fl.struct()

    fl_fin = ops.finalize_struct(GROUP, "mean_std", norm)

    def fl_step():  # the first turn fused with the restore of the reset state, the last with the finalize
        ops.frozenlake_step_turn_first(st, fl.ep, turns[0], fl.init_desc, fl.init_s, fl.init_rng)
        for t in range(1, T - 1):
            ops.frozenlake_step_turn(st, fl.ep, turns[t])
        ops.frozenlake_step_turn_finalize(st, fl.ep, turns[T - 1], fl_fin)
    fl_step()
    torch.cuda.synchronize()
    steps = int(fl.ep.turn_exec.sum().item())
    env_turns = int(fl.ep.n_turns.sum().item())
    ms = _graph_rollout(fl_step)
    gbs = env_turns * 107 / (ms * 1e-3) / 1e9  # 107 B per FrozenLake env-turn
    out["frozenlake"] = {"config": f"FrozenLake 4x4 slippery, {B} envs x {T} turns, K={K}, cap 10",
                         "env_steps_per_rollout": steps, "ms_per_rollout": ms, "env_steps_per_s": steps / ms * 1e3,
                         "env_turns_per_rollout": env_turns, "rollout_GBs": gbs, "rollout_frac": gbs / HBM_PEAK_GBS}
    # Countdown
    B, T, K = 16384, 4, 1
    inst = synthetic_instances(1024, 7)
    cd = CountdownBatch(CountdownEnvConfig(data=inst), B, T, K, device)
    cd.reset(synthetic.env_seeds(B))
    answers = synthetic.countdown_answers([inst[int(i)] for i in cd.index], T)
    bufs = []
    for t in range(T):
        lists = [[a] if a is not None else [] for a in answers[t]]
        buf, lens = cd.encode_answers(lists)
        bufs.append((torch.from_numpy(buf).to(device), torch.from_numpy(lens).to(device),
                     torch.from_numpy(np.array([len(x) for x in lists], np.uint8)).to(device)))
    zeros = torch.zeros(B, K, dtype=torch.int8, device=device)
    seg = torch.arange(0, B + 1, GROUP, dtype=torch.int32, device=device)
    norm = torch.empty(B, dtype=torch.float32, device=device)
    turns = [ops.turn_struct(t, zeros, bufs[t][2], None, 1, -0.1) for t in range(T)]
    st = cd.struct()

    def cd_step():
        cd.ep.arena.zero_()
        for t in range(T):
            ops.countdown_step_turn(st, cd.ep, turns[t], bufs[t][0], bufs[t][1])
        ops.rollout_finalize(cd.ep, seg, "mean_std", norm)
    cd_step()
    torch.cuda.synchronize()
    steps = int(cd.ep.turn_exec.sum().item())
    env_turns = int(cd.ep.n_turns.sum().item())
    ms = _graph_rollout(cd_step)
    gbs = env_turns * 159 / (ms * 1e-3) / 1e9  # 159 B per Countdown env-turn
    out["countdown"] = {"config": f"Countdown, {B} envs x {T} turns, K={K}, cap 1, 50% empty answers",
                        "env_steps_per_rollout": steps, "ms_per_rollout": ms, "env_steps_per_s": steps / ms * 1e3,
                        "env_turns_per_rollout": env_turns, "rollout_GBs": gbs, "rollout_frac": gbs / HBM_PEAK_GBS}
    return out


def text_leg(R, device, reps=20):
    """SURVEY §8(f) rank 2 on the bench's workload: the response -> action boundary on the device.
    * parse: rmi_parse_actions (_parse_response + name -> id map) over 8192 LLM-shaped
      responses of this rollout's turn-0 actions; algorithmic bytes = the text bytes read +
      the outputs (K action ids, n_actions, 4 spans) per row;
    * detokenize: rmi_detokenize over [8192, 128] token ids of a Qwen-sized (151 646) synthetic
      byte-level vocabulary; bytes = 8 per id in + the decoded bytes out;
    * text rollout: the SK rollout driven from text (5 x (parse + turn), restore and finalize
      fused, in a HIP graph) -> env-steps/s of the device-resident text API;
    * token rollout: the whole per-turn loop between two LLM generations on the device: the
      response token ids -> rmi_detok_parse (decode + parse) -> the turn -> rmi_sokoban_render (the
      next observation's text), 5 turns per rollout, in a HIP graph; and the same with the render
      fused into the turn's launch (rmi_sokoban_step_turn_render)."""
    B = R.B
    lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
    ids_h, n_h = R.ids.cpu().numpy(), R.n.cpu().numpy()
    bufs, all_texts = [], []
    for t in range(T_TURNS):
        texts = synthetic.responses_for_actions(ids_h[t], n_h[t], lk, seed=100 + t)
        all_texts.append(texts)
        buf, lens = synthetic.encode_rows(texts)
        bufs.append((torch.from_numpy(buf).to(device), torch.from_numpy(lens).to(device)))
    cfg = ops.parse_config(True, K_ACTIONS, "||", lk)
    text, tlen = bufs[0]
    for _ in range(3):
        out = ops.parse_actions(cfg, text, tlen)
    torch.cuda.synchronize()
    assert torch.equal(out["actions"], R.ids[0]) and torch.equal(out["n_actions"], R.n[0])
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        ops.parse_actions(cfg, text, tlen)
    e[1].record()
    torch.cuda.synchronize()
    parse_us = e[0].elapsed_time(e[1]) * 1e3 / reps
    text_bytes = int(((tlen.to(torch.int64) + 3) // 4 * 4).sum().item())
    pbytes = text_bytes + B * (4 + K_ACTIONS + 1 + 16)
    # detokenize
    V, Rt = 151646, 128
    rng = np.random.default_rng(5)
    lens_v = rng.integers(1, 9, size=V)
    data = rng.integers(97, 123, size=int(lens_v.sum())).astype(np.uint8)
    off = np.zeros(V + 1, np.int64)
    np.cumsum(lens_v, out=off[1:])
    skip = np.zeros(V, np.uint8)
    skip[151643:] = 1
    vt = ops.VocabTable(torch.from_numpy(off).to(device), torch.from_numpy(data).to(device),
                        torch.from_numpy(skip).to(device))
    tok = torch.from_numpy(rng.integers(0, 151643, size=(B, Rt)).astype(np.int64)).to(device)
    for _ in range(3):
        dt_out, dt_len, _ = ops.detokenize(tok, vt, 2048)
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        ops.detokenize(tok, vt, 2048)
    e[1].record()
    torch.cuda.synchronize()
    detok_us = e[0].elapsed_time(e[1]) * 1e3 / reps
    dbytes = B * Rt * 8 + int(dt_len.sum().item())
    # the rollout driven from text
    text_turns = []
    for t in range(T_TURNS):
        o = ops.parse_actions(cfg, bufs[t][0], bufs[t][1], with_spans=False)
        text_turns.append((o, ops.turn_struct(t, o["actions"], o["n_actions"], None, MAX_ACTIONS, -0.1)))

    def text_step():  # R.step()'s launches, each turn preceded by its parse
        e = R.env
        for t in range(T_TURNS):
            o, ts = text_turns[t]
            ops.parse_actions(cfg, bufs[t][0], bufs[t][1], with_spans=False, out=o)
            if t == 0:
                ops.sokoban_step_turn_first(R.st, e.ep, ts, e.init_state, e.init_player)
            elif t < T_TURNS - 1:
                ops.sokoban_step_turn(R.st, e.ep, ts)
            else:
                ops.sokoban_step_turn_finalize(R.st, e.ep, ts, R.fin)
    text_step()
    torch.cuda.synchronize()
    steps = int(R.env.ep.turn_exec.sum().item())
    ms = _graph_rollout(text_step)
    # token rollout: ids -> text -> actions -> state -> observation, every turn on the device
    table, skip = synthetic.byte_vocab()
    tvocab = ops.VocabTable.from_bytes(table, skip, device)
    tok = [torch.from_numpy(synthetic.tokenize_greedy(all_texts[t], table)).to(device) for t in range(T_TURNS)]
    stride = max(b[0].shape[1] for b in bufs)
    dec = [ops.detokenize(tok[t], tvocab, stride) for t in range(T_TURNS)]
    torch.cuda.synchronize()
    for t in range(T_TURNS):  # the decode reproduces the response texts byte for byte
        assert torch.equal(dec[t][1], bufs[t][1])
    obs = ops.sokoban_render(R.st, B, R.env.config.grid_lookup, device)
    # the fused decode + parse (rmi_detok_parse) of each turn, writing the parse outputs the
    # turn structs point at
    fused = []
    for t in range(T_TURNS):
        o, _ = text_turns[t]
        fo = ops.detok_parse(tok[t], tvocab, stride, cfg, with_spans=False)
        fused.append(dict(fo, actions=o["actions"], n_actions=o["n_actions"]))
    torch.cuda.synchronize()
    for t in range(T_TURNS):
        ops.detok_parse(tok[t], tvocab, stride, cfg, out=fused[t])
    torch.cuda.synchronize()
    for t in range(T_TURNS):  # the same text and actions as the two separate launches
        assert torch.equal(fused[t]["text_len"], bufs[t][1])
        assert torch.equal(fused[t]["actions"], R.ids[t]) and torch.equal(fused[t]["n_actions"], R.n[t])
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        ops.detok_parse(tok[0], tvocab, stride, cfg, out=fused[0])
    e[1].record()
    torch.cuda.synchronize()
    fused_us = e[0].elapsed_time(e[1]) * 1e3 / reps

    robs = ops.render_struct(R.env.config.grid_lookup, 6, 6, *obs)

    def token_step(fused_render=False):
        e = R.env
        for t in range(T_TURNS):
            o, ts = text_turns[t]
            ops.detok_parse(tok[t], tvocab, stride, cfg, out=fused[t])
            if fused_render:  # the turn renders the next observation in the same launch
                kw = {"init_state": e.init_state, "init_player": e.init_player} if t == 0 else \
                    ({"fin": R.fin} if t == T_TURNS - 1 else {})
                ops.sokoban_step_turn_render(R.st, e.ep, ts, robs, **kw)
                continue
            if t == 0:
                ops.sokoban_step_turn_first(R.st, e.ep, ts, e.init_state, e.init_player)
            elif t < T_TURNS - 1:
                ops.sokoban_step_turn(R.st, e.ep, ts)
            else:
                ops.sokoban_step_turn_finalize(R.st, e.ep, ts, R.fin)
            ops.sokoban_render(R.st, B, e.config.grid_lookup, device, out=obs)
    token_step()
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    assert int(R.env.ep.turn_exec.sum().item()) == steps
    ms_tok = _graph_rollout(token_step)
    ms_tok_fused = _graph_rollout(lambda: token_step(True))
    # one launch per turn: rmi_sokoban_token_turn (decode + parse, the turn and the render)
    tok_rows = [ops.token_rows_struct(tok[t], tvocab, cfg, fused[t]) for t in range(T_TURNS)]

    def token_turn_step():
        e = R.env
        for t in range(T_TURNS):
            _, ts = text_turns[t]
            kw = {"init_state": e.init_state, "init_player": e.init_player} if t == 0 else \
                ({"fin": R.fin} if t == T_TURNS - 1 else {})
            ops.sokoban_token_turn(tok_rows[t], R.st, e.ep, ts, robs, **kw)
    token_turn_step()
    torch.cuda.synchronize()
    assert int(R.env.ep.turn_exec.sum().item()) == steps
    ms_tok_one = _graph_rollout(token_turn_step)
    # render alone
    torch.cuda._sleep(2_000_000)
    e[0].record()
    for _ in range(reps):
        ops.sokoban_render(R.st, B, R.env.config.grid_lookup, device, out=obs)
    e[1].record()
    torch.cuda.synchronize()
    render_us = e[0].elapsed_time(e[1]) * 1e3 / reps
    return {"parse": {"kernel": "rmi_parse_actions", "rows": B, "text_bytes": text_bytes, "us": parse_us,
                      "achieved_GBs": pbytes / (parse_us * 1e-6) / 1e9,
                      "frac": pbytes / (parse_us * 1e-6) / 1e9 / HBM_PEAK_GBS},
            "detokenize": {"kernel": "rmi_detokenize", "rows": B, "ids_per_row": Rt, "vocab": V, "us": detok_us,
                           "achieved_GBs": dbytes / (detok_us * 1e-6) / 1e9,
                           "frac": dbytes / (detok_us * 1e-6) / 1e9 / HBM_PEAK_GBS},
            "text_rollout": {"config": "SK rollout from response text: 5 x (parse + turn), restore and finalize fused",
                             "env_steps_per_rollout": steps, "ms_per_rollout": ms,
                             "env_steps_per_s": steps / ms * 1e3},
            "detok_parse": {"kernel": "rmi_detok_parse", "rows": B, "ids_per_row": int(tok[0].shape[1]),
                            "vocab": "byte-level (synthetic.byte_vocab)", "us": fused_us,
                            "note": "the decode fused with the parse: one launch per turn on the token path"},
            "token_rollout": {"config": "SK rollout from response token ids: 5 x rmi_sokoban_token_turn (decode + "
                                        "parse, turn and render in one launch per turn)",
                              "env_steps_per_rollout": steps, "ms_per_rollout": ms_tok_one,
                              "env_steps_per_s": steps / ms_tok_one * 1e3,
                              "ms_per_rollout_three_launches": ms_tok,
                              "ms_per_rollout_turn_render_fused": ms_tok_fused,
                              "note": "three launches: detok_parse, the turn, the render per turn; "
                                      "turn_render_fused: detok_parse, then rmi_sokoban_step_turn_render (DESIGN 3.10)"},
            "render": {"kernel": "rmi_sokoban_render", "envs": B, "us": render_us}}


def prompt_kernels(proxy, tok, device, turn=2, reps=10):
    """the caller path's text kernels on the API rollout's own rows (the last
    rollout's turn-``turn`` slot of the turn chain, 8192 envs), relaunched alone with HIP events:
    * prompt_text (rmi_prompt_text): the assistant + user block text of every row; bytes = the
      decoded responses and observation rows read + the text written;
    * bpe_encode (rmi_bpe_encode): that text -> ids at the chain's row bound; bytes = text in + 8 B
      per id out (word cache warm; also one launch with it cleared);
    * pad_rows (rmi_pad_rows): the generation batch of the final turn (every env's arena row,
      left-padded to the widest + the generation prompt); bytes = 8 B per arena id read + 3 x 8 B
      per output cell;
    * bpe_merge_table: the same turn's text built on the host (no expansion placeholders: every
      template byte is encoded) through the 5 k-merge tokenizer and through a Qwen2-sized one
      (synthetic.qwen_scale_tokenizer, 151 000 merges), ids checked against the HF tokenizers."""
    from ragen_amd.tokenizer import DeviceTokenizer
    es = proxy.train_es_manager
    ch = es.__dict__.get("_chain")
    if ch is None or turn not in ch.slots or ch.slots[turn].prompt is None:
        return None
    s, pr, n = ch.slots[turn], ch.pr, es.n_envs
    L = _lib.lib()
    stream = ops._stream(device)
    _, _, pstride, bound, _, held = s.prompt
    P = ctypes.byref(held[0])  # the turn's rmi_prompt_t
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(fn, r=reps):
        fn()
        torch.cuda.synchronize()
        torch.cuda._sleep(1_000_000)
        ev[0].record()
        for _ in range(r):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) * 1e3 / r

    def blk(us, nbytes, **kw):
        gbs = nbytes / (us * 1e-6) / 1e9
        return dict(kw, us=us, bytes=int(nbytes), achieved_GBs=gbs, frac=gbs / HBM_PEAK_GBS)

    out = {"rows": n, "turn": turn}
    # prompt_text
    pt_us = timed(lambda: ops.check(L.rmi_prompt_text(P, n, s.ptext.data_ptr(), pstride, s.ptext_len.data_ptr(),
                                                      s.pmark.data_ptr(), s.pterr.data_ptr(), stream),
                                    "rmi_prompt_text"))
    act = s.has.bool()
    resp_b = int(s.tlen[act].to(torch.int64).sum())
    obs_b = int(s.obs[1][act].to(torch.int64).sum())
    text_b = int(s.ptext_len.to(torch.int64).sum())
    out["prompt_text"] = blk(pt_us, resp_b + obs_b + text_b, kernel="rmi_prompt_text", text_bytes_out=text_b)
    # bpe_encode
    dt = pr.dt
    bs = dt.bpe_struct()
    ids = torch.zeros(n, 2048, dtype=torch.int64, device=device)
    olen = torch.zeros(n, dtype=torch.int32, device=device)
    ntok = torch.empty(n, dtype=torch.int32, device=device)
    mtok = torch.empty(n, dtype=torch.int32, device=device)
    err = torch.empty(n, dtype=torch.uint8, device=device)

    def bpe():
        ops.check(L.rmi_bpe_encode(ctypes.addressof(bs), s.ptext.data_ptr(), pstride, bound, s.ptext_len.data_ptr(),
                                   n, ids.data_ptr(), 2048, None, ntok.data_ptr(), s.pmark.data_ptr(),
                                   mtok.data_ptr(), err.data_ptr(), stream), "rmi_bpe_encode")
    bpe_us = timed(bpe)
    n_ids = int(ntok.to(torch.int64).sum())
    assert int((err != 0).sum()) == 0
    cold = None
    if dt.word_cache is not None:
        saved = dt.word_cache.clone()
        dt.word_cache.zero_()
        cold = timed(bpe, 1)
        dt.word_cache.copy_(saved)
    out["bpe_encode"] = blk(bpe_us, text_b + 8 * n_ids, kernel="rmi_bpe_encode", row_bound=bound, ids_out=n_ids,
                            text_GBs=text_b / (bpe_us * 1e-6) / 1e9, us_word_cache_cleared=cold,
                            note="the chain's text: template stretches as expansion placeholders (their ids "
                                 "copied, their bytes not encoded)")
    # pad_rows: the final turn's generation batch shape over every env
    S = int(pr.len.max()) + pr.tail_n
    rows = torch.arange(n, dtype=torch.int64, device=device)
    pad = torch.empty(3, n, S, dtype=torch.int64, device=device)
    perr = torch.empty(n, dtype=torch.uint8, device=device)
    pad_us = timed(lambda: ops.check(L.rmi_pad_rows(pr.arena_p, pr.arena_stride, pr.len_p, rows.data_ptr(), n,
                                                    pr.tail_p, pr.tail_n, S, int(pr.pad_id), pad[0].data_ptr(),
                                                    pad[1].data_ptr(), pad[2].data_ptr(), perr.data_ptr(), stream),
                                    "rmi_pad_rows"))
    arena_ids = int(pr.len.to(torch.int64).sum()) + n * pr.tail_n
    out["pad_rows"] = blk(pad_us, 8 * arena_ids + 24 * n * S, kernel="rmi_pad_rows", width=S)
    del pad
    # the merge-table size: the same turn's text from the host, both tokenizers
    texts = []
    has_h, fl_h = s.has.cpu().numpy(), s.flags_copy.cpu().numpy()
    for e in np.flatnonzero(has_h):
        a, b = pr.host_turn_text(int(e), turn, not (int(fl_h[e]) & _lib.FLAG_DONE))
        texts.append(a + b)
    buf, lens = synthetic.encode_rows(texts)
    tb = torch.from_numpy(buf).to(device)
    tl = torch.from_numpy(lens).to(device)
    stride = min(3072, (int(lens.max()) + 3) // 4 * 4)
    big = synthetic.qwen_scale_tokenizer(base=tok)
    res = {"rows": len(texts), "text_bytes": int(lens.sum()), "row_bound": stride}
    for name, t in (("merges_5k", tok), ("merges_151k", big)):
        d = DeviceTokenizer.from_hf(t, device)
        o = torch.zeros(len(texts), 2048, dtype=torch.int64, device=device)
        oln = torch.zeros(len(texts), dtype=torch.int32, device=device)

        def enc():
            oln.zero_()
            return d.encode_rows(tb, tl, o, oln, max_len=stride)
        n_tok, _, e8 = enc()
        torch.cuda.synchronize()
        assert int((e8 != 0).sum()) == 0
        for i in range(0, len(texts), max(1, len(texts) // 64)):  # ids == the HF tokenizer's, 64 rows
            want = t(texts[i], add_special_tokens=False).input_ids
            assert o[i, :int(n_tok[i])].tolist() == want, (name, i)
        us = timed(lambda: enc())
        cold_us = None
        if d.word_cache is not None:
            d.word_cache.zero_()
            cold_us = timed(lambda: enc(), 1)
        merges = int(len(json.loads(t.backend_tokenizer.to_str())["model"]["merges"]))
        res[name] = {"merges": merges, "us": us, "us_word_cache_cleared": cold_us,
                     "ids_out": int(n_tok.to(torch.int64).sum()),
                     "text_GBs": int(lens.sum()) / (us * 1e-6) / 1e9}
    res["ratio_151k_to_5k"] = res["merges_151k"]["us"] / res["merges_5k"]["us"]
    res["ratio_151k_to_5k_cold"] = (res["merges_151k"]["us_word_cache_cleared"] /
                                    res["merges_5k"]["us_word_cache_cleared"])
    out["bpe_merge_table"] = res
    return out


def api_leg(device):
    """SURVEY §8(d)'s "API" variant of the headline: the same SK workload (8192 envs, 5 turns, the
    bench's synthetic actions written as LLM responses) driven through the drop-in
    LLMAgentProxy.rollout (agent_proxy.py:143-159), reset excluded, with a Qwen2-pipeline
    byte-level BPE tokenizer (synthetic.qwen_like_tokenizer: the Qwen2.5 tokenizer is a hub
    download) and an actor that reads the prompt batch every turn, as a vLLM worker group does
    (input_ids / attention_mask / position_ids, agent_proxy.py:128-141):
    * ``device`` path — responses arrive as token ids on the GPU; the ContextManager decodes
      them on the device, EnvStateManager parses, steps and renders on the device, and the
      prompt ids of the next turn are built and tokenized on the device (llm_agent/prompts.py);
      ``env_steps_per_s`` = env steps / (turn loop + get_rollout_states + formulate_rollouts),
      every phase of the rollout after the reset;
    * ``dict`` path — EnvStateManager.step fed the reference's list of dicts with action names
      (per-turn device round trip, host history dicts and text observations each turn)."""
    import random
    from ragen_amd.config import env_task
    from ragen_amd.llm_agent import EnvStateManager, LLMAgentProxy, TokenActor
    from ragen_amd.protocol import DataProto
    B, T, K = B_PER_GPU, T_TURNS, K_ACTIONS
    cfg = env_task("SimpleSokoban", B // GROUP, GROUP, max_turn=T, max_actions_per_turn=K)
    ids, n = synthetic.rollout_actions(B, T, K, 1, 4)
    lk = {1: "Up", 2: "Down", 3: "Left", 4: "Right"}
    tok = synthetic.qwen_like_tokenizer()
    tokens = []
    for t in range(T):
        enc = tok(synthetic.responses_for_actions(ids[t], n[t], lk, seed=100 + t), padding=False).input_ids
        R = max(len(x) for x in enc)
        a = np.full((B, R), tok.pad_token_id, np.int64)
        for i, x in enumerate(enc):
            a[i, :len(x)] = x
        tokens.append(torch.from_numpy(a).to(device))
    actor = TokenActor(tokens, read_prompts=True)
    proxy = LLMAgentProxy(cfg, actor, tok, device=device)
    proxy.train_ctx_manager.set_device_vocab(ops.VocabTable.from_tokenizer(tok, device))
    runs = []
    random.seed(0)  # one train-seed sequence, as a training loop draws it (reset() prefetches the next rooms)
    for rep in range(4):
        actor.turn = 0
        actor.prompts, actor.prompt_shapes = [], []
        torch.cuda.synchronize()
        out = proxy.rollout(DataProto(meta_info={}), val=False)
        torch.cuda.synchronize()
        steps = int(proxy.train_es_manager.tags[0].batch.ep.turn_exec.sum().item())
        runs.append((steps, dict(proxy.last_timing), len(out), list(actor.prompt_shapes),
                     tuple(out.batch["input_ids"].shape),
                     bool(getattr(proxy.train_es_manager.tags[0].batch, "reset_prefetched", False))))
    pr = proxy.train_ctx_manager.prompts()
    steps, tm, rows, shapes, upd, prefetched = runs[-1]
    total = tm["turns_s"] + tm["rollout_states_s"] + tm["formulate_s"]
    device_path = {"env_steps": steps, "turn_loop_s": tm["turns_s"], "get_rollout_states_s": tm["rollout_states_s"],
                   "formulate_rollouts_s": tm["formulate_s"], "rollout_s": total, "env_steps_per_s": steps / total,
                   "turn_loop_env_steps_per_s": steps / tm["turns_s"], "rows_formulated": rows,
                   "reset_s": tm["reset_s"],  # es.reset(): rooms for a fresh train seed (host) + device restore
                   "reset_rooms_prefetched": prefetched,  # generated behind the previous rollout (SokobanBatch.prefetch)
                   "env_steps_per_s_with_reset": steps / (total + tm["reset_s"]),
                   "readbacks": tm.get("readbacks"), "turns": len(shapes),
                   "eager_prompt_turns": pr.eager_turns if pr is not None else None,
                   "chain_padded_batches": pr.chain_padded if pr is not None else None,  # (4 rollouts)
                   "prompt_batch_shapes": shapes, "update_batch_shape": upd, "device_prompts": pr is not None,
                   "host_prompt_rows": pr.host_rows_used if pr is not None else None,
                   "tokenizer": f"{tok.name_or_path}, vocab {len(tok)}",
                   "note": "LLMAgentProxy.rollout, response token ids on the GPU, an actor reading input_ids / "
                           "attention_mask / position_ids every turn, device prompt ids; last of 4 rollouts"}
    # the dict facade: EnvStateManager.step with the reference's list-of-dict inputs, the turn
    # reaching the kernel through the torch custom op (the facade's default) and through ctypes
    from ragen_amd.env import SokobanBatch
    names = {1: "Up", 2: "Down", 3: "Left", 4: "Right", 0: "Jump"}  # 0 = a name outside the action lookup
    turn_inputs = [[[names[int(a)] for a in ids[t, i, :int(n[t, i])]] for i in range(B)] for t in range(T)]

    def dict_rollout():
        es = EnvStateManager(cfg, mode="train", device=device)
        es.reset(seed=synthetic.ENV_SEED)
        active = list(range(B))
        dsteps = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(T):
            inputs = [{"env_id": i, "llm_response": "", "llm_raw_response": "", "actions": turn_inputs[t][i]}
                      for i in active]
            outs = es.step(inputs)
            active = [o["env_id"] for o in outs]
            dsteps += int(es.tags[0].batch.ep.turn_exec[t].sum().item())
            if not active:
                break
        return dsteps, time.perf_counter() - t0

    dict_path = {}
    import gc
    runs = {"op": [], "ctypes": []}
    try:  # the two routes alternate (host noise hits both alike); best of 4 each
        for _ in range(4):
            for mode in ("op", "ctypes"):
                SokobanBatch.dispatch = mode
                gc.collect()
                runs[mode].append(dict_rollout())
    finally:
        SokobanBatch.dispatch = "op"
    for mode in ("op", "ctypes"):
        dsteps, dt = min(runs[mode], key=lambda r: r[1])
        dict_path[mode] = {"env_steps": dsteps, "seconds": dt, "env_steps_per_s": dsteps / dt}
    # the per-call host cost of the two dispatch routes (one 8192-env turn launch, no env acting)
    env = SokobanBatch(None, B, T, K, device)
    z8 = torch.zeros(B, K, dtype=torch.int8, device=device)
    zu = torch.zeros(B, dtype=torch.uint8, device=device)
    per_call = {}
    for mode in ("op", "ctypes"):
        env.dispatch = mode
        for _ in range(20):
            env.step_turn(0, z8, zu, zu, 10, -0.1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(500):
            env.step_turn(0, z8, zu, zu, 10, -0.1)
        per_call[mode] = (time.perf_counter() - t0) / 500 * 1e6
        torch.cuda.synchronize()
    prompt = prompt_kernels(proxy, tok, device)
    return {"env_steps_per_s": device_path["env_steps_per_s"], "device_path": device_path, "prompt_kernels": prompt,
            "dict_path": dict(dict_path["op"], ctypes=dict_path["ctypes"], host_us_per_turn_call=per_call,
                              note="EnvStateManager.step facade, host dicts + text obs each turn (the action-name "
                                   "lists are built before the timed loop); best of 4 rollouts; the top level "
                                   "goes through the torch custom op, `ctypes` through the C ABI directly")}


def host_cpus():
    """The host cores this process may use: the affinity mask, capped by the box's CPU share
    (OMP_NUM_THREADS is set to it on the GPU box, where nproc shows the whole machine), plus the
    machine's nproc and CPU model (SURVEY §8(d) asks for both)."""
    aff = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    cores = min(aff, int(share)) if share and share.isdigit() and int(share) > 0 else aff
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cores": cores, "affinity": aff, "omp_num_threads": share, "nproc": os.cpu_count(), "model": model}


def cpu_baseline_parallel(R, workers=None, reps=20):
    """SURVEY §8(d) CPU baseline (b): one process per host core (host_cpus(): the affinity
    mask capped by the box's share), env groups partitioned across processes, no shared state.
    Worker w runs ``reps`` rollouts of the 2048-env slice (w % 4) of this rank's batch; value =
    all workers' env steps / wall time of the parallel phase (process start-up excluded)."""
    import multiprocessing as mp
    from oracle import port
    hc = host_cpus()
    workers = workers or hc["cores"]
    n_envs = 2048
    jobs = []
    for w in range(workers):
        lo = (w % (B_PER_GPU // n_envs)) * n_envs
        sl = slice(lo, lo + n_envs)
        jobs.append((R.env.room_fixed[sl].cpu().numpy(), R.env.init_state[sl].cpu().numpy(),
                     R.env.init_player[sl].cpu().numpy(), R.ids[:, sl].cpu().numpy(), R.n[:, sl].cpu().numpy(),
                     MAX_ACTIONS, reps))
    ctx = mp.get_context("spawn")  # a child process per worker (no fork of this GPU process)
    with ctx.Pool(workers) as pool:
        pool.map(abs, range(workers))  # workers started and warm
        t0 = time.perf_counter()
        res = pool.starmap(port.timed_rollouts, jobs)
        wall = time.perf_counter() - t0
    steps = sum(r[0] for r in res)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": workers, "kind": "port", "host": hc,
            "sample": f"{workers} processes x {reps} rollouts of {n_envs} envs x {T_TURNS} turns, {steps} env.step "
                      f"calls in {wall:.1f}s wall, oracle/port.py"}


def cpu_gae_baseline(R, reps=2):
    """the advantage step as the reference runs it — verl GAE (legacy, a Python
    loop over token columns, torch on the host) + masked whitening (oracle/port.py) — on the
    same token rows as the `advantage` leg, with 1 thread and with 16.  -> tokens/s each."""
    from oracle import port
    n_turns = R.env.ep.n_turns.cpu().numpy()
    score = R.norm.cpu().numpy()
    r, v, m = (torch.from_numpy(x) for x in synthetic.token_rows(n_turns, score, seed=11))
    out = {"kind": "port", "rows": int(r.shape[0]), "cols": int(r.shape[1]),
           "sample": "verl compute_gae_advantage_return (legacy) + masked_whiten on the advantage leg's rows, "
                     f"best of {reps}"}
    old = torch.get_num_threads()
    many = host_cpus()["cores"]
    out["threads"] = [1, many]
    try:
        for threads in (1, many):
            torch.set_num_threads(threads)
            best = None
            for _ in range(reps):
                t0 = time.perf_counter()
                port.verl_gae_whiten(r, v, m, 1.0, 1.0)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            out[f"tokens_per_s_{threads}t"] = r.numel() / best
            out[f"ms_{threads}t"] = best * 1e3
    finally:
        torch.set_num_threads(old)
    return out


def cpu_baseline(R, seconds_budget=20.0):
    """Reference-shaped CPU path (oracle/port.py: per-env Python objects mirroring
    EnvStateManager.step + SokobanEnv.step) on a bounded sample of the same workload:
    the first n_envs envs of this rank's batch, same rooms, same synthetic actions."""
    from oracle import port
    n_envs = 2048
    fixed = R.env.room_fixed[:n_envs].cpu().numpy()
    state0 = R.env.init_state[:n_envs].cpu().numpy()
    player0 = R.env.init_player[:n_envs].cpu().numpy()
    ids = R.ids[:, :n_envs].cpu().numpy()
    n = R.n[:, :n_envs].cpu().numpy()
    steps = 0
    reps = 0
    dt = 0.0
    while True:
        envs = port.make_sokoban_envs(fixed, state0, player0)
        t0 = time.perf_counter()
        steps += port.sokoban_rollout(envs, ids, n, MAX_ACTIONS)
        dt += time.perf_counter() - t0
        reps += 1
        if dt > seconds_budget / 2 or reps >= 40:
            break
    return {"value": steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port", "host": host_cpus(),
            "sample": f"{reps} x Sokoban 6x6 rollout of {n_envs} envs x {T_TURNS} turns (reset excluded), "
                      f"{steps} env.step calls in {dt:.1f}s, 1 thread, oracle/port.py"}


def launch_plan(gpus, environ, device_count):
    """How this invocation runs, decided before anything touches the GPU.
    -> ("run", world)            : this process is one rank of `world` (torchrun set WORLD_SIZE,
                                   or a plain N=1 run);
       ("spawn", gpus)           : `python bench.py --gpus N` with no launcher: start N rank
                                   processes (torch.distributed.run, 127.0.0.1) and exit with
                                   their status;
       ("error", message)        : the request cannot be honoured (fewer devices than ranks, or
                                   a launcher world that disagrees with --gpus) -> exit non-zero,
                                   never a silently relabelled 1-GPU run."""
    if gpus < 1:
        return "error", f"--gpus {gpus}: need at least 1"
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        if gpus == 1:
            return "run", 1
        if device_count < gpus:
            return "error", (f"--gpus {gpus} asks for {gpus} ranks, one per GPU, but this box has {device_count} "
                             "GPU(s); RCCL does not place two ranks on one device (use --double-buffer to run the "
                             "N>1 exchange path as a 1-rank group on one GPU)")
        return "spawn", gpus
    world = int(ws)
    if world != gpus:
        return "error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"
    local = int(environ.get("LOCAL_RANK", "0"))
    if local >= device_count:
        return "error", f"LOCAL_RANK {local} has no device (this box has {device_count} GPU(s))"
    return "run", world


def exchange_plan(mode, per_gather, G):
    """The N>1 exchange placement: -> (mode, rollouts per gather).  The default is StarPO's own
    order (agent_trainer.py:514-655): every rollout's record all-gathered right after it, serial
    on the critical path, because the gathered batch feeds compute_advantage and the update
    before the next rollout starts.  A gather per several rollouts (per_gather > 1) or the
    overlapped placement (a gather behind the NEXT rollouts, which training cannot do) are
    extras; overlap always gathers a whole replay's G rollouts."""
    per_gather = int(per_gather)
    if per_gather < 1:
        raise ValueError("--rollouts-per-gather must be >= 1")
    if mode == "serial":
        if G % per_gather:
            raise ValueError(f"--rollouts-per-gather {per_gather} must divide the {G} rollouts of a graph replay")
        return "serial", per_gather
    return mode, G  # overlap / auto: the amortised placements (auto picks between them)


def serial_exchange(step, chunk, outs, G, p, gather=None):
    """G rollouts on one stream, each run of p followed by its all-gather (step(j) runs rollout
    j; chunk(p, k) is the k-th run of p arenas; outs[k] its gathered bytes): with p = 1 every
    rollout's record is reassembled before the next rollout starts, the StarPO order."""
    gather = gather or rd.gather_bytes
    for j in range(G):
        step(j)
        if (j + 1) % p == 0:
            k = j // p
            gather(chunk(p, k), outs[k])


def setup_ipc_exchange(nbytes, device, src, probes=4):
    """The one-shot exchange (ragen_amd.exchange) for this rank's arena of nbytes, checked before
    use: `probes` eager exchanges of src, each gathered slot checked with check_gathered (every
    rank's row against the digest its owner all-gathered).  Collective.  -> (ArenaExchange or
    None, reason): None on every rank when any rank failed the setup or a probe (the caller
    then gathers with RCCL)."""
    from ragen_amd import exchange as xgm
    try:
        xg = xgm.ArenaExchange(nbytes, device)
    except Exception as ex:  # raised on every rank alike (the setup agrees after each step)
        return None, f"setup failed: {ex}"
    ok, why = True, ""
    try:
        g = torch.Generator(device="cpu").manual_seed(7919 + xg.rank)
        for _ in range(probes):  # rank-distinct bytes: a row landing in the wrong place fails
            src.copy_(torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g))
            xg.run(src)
            ok = check_gathered(src.reshape(-1), xg.slot().contiguous().view(-1), xg.world, xg.rank,
                                distinct=True) and ok
        torch.cuda.synchronize()
        err = xg.error()
        ok = ok and err == 0
        why = f"probe: rows {'ok' if ok else 'WRONG'}, err bits {err}"
    except Exception as ex:
        ok, why = False, f"probe raised: {ex}"
    if not xgm.agree(ok):
        tdist.barrier()
        xg.close()
        return None, why or "probe failed on another rank"
    xg.sync_epoch()
    return xg, why


def exchange_label(mode, P, G, asked, graph, transport="rccl"):
    if transport == "ipc" and graph and mode == "serial" and P == 1:
        return ("one-shot exchange of the episode arena after every rollout, serial on the same stream (StarPO "
                "order): every rank stores its arena into every rank's IPC-mapped region, one launch")
    if not graph:
        return "all-gather of the episode arena after every rollout, serial (eager)"
    if mode == "overlap":
        return (f"one all-gather per {G} rollouts, overlapped with the next {G} on a comm stream "
                f"(amortised extra; --exchange {asked})")
    if P == 1:
        return "all-gather of the episode arena after every rollout, serial on the same stream (StarPO order)"
    return f"one all-gather per {P} rollouts, serial on the same stream (amortised extra; --exchange {asked})"


def spawn_ranks(gpus, argv):
    """Start `gpus` rank processes of this script through torch.distributed.run on 127.0.0.1 (a
    free port), wait, and return their exit status.  The parent never initialises the GPU."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def arena_digests(sets):
    """u8[R, n] (R rows: one rank's arena set per row) -> i64[R] digests: a position-weighted
    sum of the row's 32-bit words (exact mod 2^64, so independent of reduction order).  A rank
    broadcasts the digest of its own set; every rank recomputes the digests of the gathered rows
    and compares, so a garbage or misplaced row of ANY rank fails the check."""
    R, n = sets.shape
    pad = (-n) % 4
    x = sets if pad == 0 else torch.cat([sets, sets.new_zeros(R, pad)], 1)
    w = x.contiguous().view(torch.int32).to(torch.int64)
    k = torch.arange(w.shape[1], dtype=torch.int64, device=sets.device)
    weight = (k * 2654435761 + 40503) % 2147483647 + 1
    return (w * weight).sum(1)


def check_gathered(own, gathered, world, rank, distinct=True):
    """The N>1 exchange check of one gathered arena set (collective: every rank calls it).
    own: u8[n] this rank's set; gathered: u8[world * n] the all-gather's result.  Every rank
    all-gathers the digest of its own set, then checks every row of its gathered copy against
    those digests, and its own row byte for byte.  distinct: the ranks' sets differ (they seed
    different groups), so a row copied from another rank also fails.  -> bool (this rank)."""
    rows = gathered.view(world, -1)
    every = torch.empty(world, dtype=torch.int64, device=own.device)
    tdist.all_gather_into_tensor(every, arena_digests(own.reshape(1, -1)))
    ok = torch.equal(rows[rank], own.reshape(-1)) and torch.equal(arena_digests(rows), every)
    if distinct and world > 1:
        ok = ok and int(torch.unique(every).numel()) == world
    return bool(ok)


def make_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the advantage leg and the copy-peak probe")
    ap.add_argument("--group", type=int, default=8, help="rollouts per graph replay (reduced to divide --steps)")
    ap.add_argument("--exchange", choices=("serial", "overlap", "auto"), default="serial",
                    help="N>1: the all-gather serial after its rollouts on the same stream (StarPO: the gathered "
                         "batch feeds compute_advantage and the update before the next rollout), or overlapped "
                         "with the next rollouts on a comm stream (an extra: training cannot do that)")
    ap.add_argument("--rollouts-per-gather", type=int, default=1,
                    help="N>1: rollouts whose arenas one all-gather reassembles (1 = every rollout's batch "
                         "gathered before its update, as agent_trainer.fit does; >1 amortises it: an extra)")
    ap.add_argument("--double-buffer", action="store_true",
                    help="run the N>1 exchange path at N=1 (a 1-rank RCCL group, real collectives)")
    ap.add_argument("--no-boards", action="store_true",
                    help="turn launches without the board cache (every turn decodes the grid rows; A/B)")
    ap.add_argument("--transport", choices=("auto", "ipc", "rccl"), default="auto",
                    help="N>1: how the per-rollout arena gather moves bytes: 'ipc' = the one-shot exchange "
                         "(every rank stores its arena into every peer's IPC-mapped region, rmi_xgather), 'rccl' = "
                         "RCCL's all-gather; 'auto' = ipc when its setup and probe pass on every rank, else rccl")
    return ap


def main():
    args = make_parser().parse_args()

    # torch.cuda.device_count() does not initialise the GPU on this image, so the parent of a
    # self-spawned run stays GPU-free
    action, what = launch_plan(args.gpus, os.environ, torch.cuda.device_count())
    if action == "error":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if action == "spawn":
        sys.exit(spawn_ranks(what, sys.argv[1:]))
    world = what
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1 or args.double_buffer
    torch.cuda.set_device(local)  # before the process group: RCCL binds its communicator to this device
    device = torch.device("cuda", local)
    if dist:
        if world == 1:  # --double-buffer at N=1: a 1-rank RCCL group exercises the N>1 path
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29517"), ("RANK", "0"), ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)
        tdist.init_process_group("nccl", device_id=device)

    R = Rollout(device, rank, boards=not args.no_boards)
    # env steps per rollout (deterministic: every replay executes the same actions)
    R.step()
    torch.cuda.synchronize()
    steps_per_rollout = int(R.env.ep.turn_exec.sum().item())
    # active envs per launch = envs stepped in that turn (n_turns > t)
    n_turns = R.env.ep.n_turns.cpu().numpy()
    active_per_turn = [int((n_turns > t).sum()) for t in range(T_TURNS)]

    # Graph replay, G rollouts per replay (G = --group, reduced until it divides --steps; every
    # rollout is a full restore (fused into turn 0) + T turns + finalize into its own episode arena).
    # N > 1: the rollout's real exchange step (north_star) — reassemble every
    # rank's trajectory record before the PPO update — is ONE RCCL all-gather of the G arenas of
    # a replay (they are contiguous: EpisodeState.pool), captured in its own graph and replayed
    # on a comm stream, so it overlaps the next G rollouts.  Two arena sets alternate; a set is
    # rewritten only after its previous gather finished (events).  Multi-stream capture and one
    # event pair per rollout were both measured slower (tools/overlap_probe.py).
    G = 1
    for g in (args.group, 8, 4, 2, 1):
        if 1 <= g <= args.group and args.steps % g == 0:
            G = g
            break
    exchange_mode, P = exchange_plan(args.exchange, args.rollouts_per_gather, G) if dist else (None, 1)

    def capture(fn, stream=None):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            fn()
        return g

    graph = None
    variants = None
    transport, xg, xg_note = ("rccl" if dist else None), None, None
    if not args.no_graph:
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            for _ in range(3):
                R.step()
        torch.cuda.current_stream(device).wait_stream(s)
        pool, eps = ops.EpisodeState.pool(2 * G, R.env.B, R.env.T, device)
        sets = pool.view(2, -1)  # set h = arenas [h*G, (h+1)*G), contiguous

        def rollouts(h):
            for j in range(G):
                R.env.ep = eps[h * G + j]
                R.step()

        roll_g = [capture(lambda h=h: rollouts(h)) for h in (0, 1)]
        R.env.ep = eps[0]
        graph = roll_g[0]
        main_s = torch.cuda.current_stream(device)
        count = [0]
        if not dist:
            def run():
                roll_g[(count[0] // G) & 1].replay()
                count[0] += G
        else:
            W = tdist.get_world_size()
            arena_bytes = sets.shape[1] // G
            # outs[p][h][k]: the gathered bytes of set h's k-th chunk of p rollouts (p = 1: every
            # rollout's arena on its own, the StarPO headline; p = G: one gather per replay)
            outs = {p: [[torch.empty(W * p * arena_bytes, dtype=torch.uint8, device=device) for _ in range(G // p)]
                        for _ in (0, 1)] for p in sorted({1, G})}

            def chunk(h, p, k):  # set h's k-th run of p contiguous arenas
                return sets[h][k * p * arena_bytes:(k + 1) * p * arena_bytes]

            comm, cap_s = torch.cuda.Stream(device), torch.cuda.Stream(device)
            comm.wait_stream(main_s)
            with torch.cuda.stream(comm):  # communicator setup must not happen under capture
                for p in outs:
                    for h in (0, 1):
                        for k in range(G // p):
                            rd.gather_bytes(chunk(h, p, k), outs[p][h][k])
            torch.cuda.synchronize()

            def serial_body(h, p):
                def step(j):
                    R.env.ep = eps[h * G + j]
                    R.step()
                serial_exchange(step, lambda q, k: chunk(h, q, k), outs[p][h], G, p)

            serial_g = {p: [capture(lambda h=h, p=p: serial_body(h, p)) for h in (0, 1)] for p in outs}
            # the one-shot exchange (ipc): every rollout's arena stored into every rank's region
            # by one launch right after the rollout, on the same stream (the StarPO order)
            xg, xg_note = None, "--transport rccl"
            if args.transport != "rccl":
                xg, xg_note = setup_ipc_exchange(arena_bytes, device,
                                                 torch.empty(arena_bytes, dtype=torch.uint8, device=device))
                if xg is None and args.transport == "ipc":
                    raise RuntimeError(f"--transport ipc: {xg_note}")
            transport = "ipc" if xg is not None else "rccl"
            if xg is not None:
                def ipc_body(h):
                    def step(j):
                        R.env.ep = eps[h * G + j]
                        R.step()
                    serial_exchange(step, lambda q, k: chunk(h, q, k), [None] * G, G, 1,
                                    gather=lambda src, out: xg.run(src))

                ipc_g = [capture(lambda h=h: ipc_body(h)) for h in (0, 1)]
                xg.sync_epoch()  # (capture recorded the launches without running them)

                def run_ipc():
                    ipc_g[(count[0] // G) & 1].replay()
                    count[0] += G
                    xg.advance(G)
            gather_g = [capture(lambda h=h: rd.gather_bytes(sets[h], outs[G][h][0]), stream=cap_s) for h in (0, 1)]
            R.env.ep = eps[0]
            rolled = [torch.cuda.Event(), torch.cuda.Event()]
            gathered = [torch.cuda.Event(), torch.cuda.Event()]

            def run_overlap():  # amortised: one gather per G rollouts, behind the next G (an extra)
                h = (count[0] // G) & 1
                if count[0] >= 2 * G:
                    main_s.wait_event(gathered[h])  # set h's previous gather has read it
                roll_g[h].replay()
                rolled[h].record(main_s)
                torch.cuda.set_stream(comm)
                comm.wait_event(rolled[h])
                gather_g[h].replay()
                gathered[h].record(comm)
                torch.cuda.set_stream(main_s)
                count[0] += G

            def run_serial_p(p):
                def run_s():
                    serial_g[p][(count[0] // G) & 1].replay()
                    count[0] += G
                return run_s

            def trial(fn, n=4):
                tdist.barrier()
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(n):
                    fn()
                torch.cuda.synchronize()
                dt = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=device)
                tdist.all_reduce(dt, op=tdist.ReduceOp.MAX)  # every rank picks the same mode
                return float(dt.item())

            if exchange_mode == "auto":  # amortised placements only (P = G): which wins depends on W
                t_ov = min(trial(run_overlap) for _ in range(3))
                t_se = min(trial(run_serial_p(G)) for _ in range(3))
                exchange_mode = "overlap" if t_ov <= t_se else "serial"
            run = run_overlap if exchange_mode == "overlap" else run_serial_p(P)
            if transport == "ipc" and exchange_mode == "serial" and P == 1:
                run = run_ipc
                if args.transport == "auto":  # the faster of the two transports on this node
                    t_ipc = min(trial(run_ipc) for _ in range(3))
                    t_rccl = min(trial(run_serial_p(1)) for _ in range(3))
                    xg_note = (f"{xg_note}; auto: one-shot {t_ipc / (4 * G) * 1e3:.4f} ms vs RCCL "
                               f"{t_rccl / (4 * G) * 1e3:.4f} ms per rollout (best of 3 trials, max over ranks)")
                    if t_rccl < t_ipc:
                        run, transport = run_serial_p(1), "rccl"
            else:
                transport = "rccl"  # (the amortised placements gather with RCCL)

            def variants_fn():
                """ms per rollout of every placement, max over ranks, best of 3 trials of 4 replays
                each: the StarPO form (a gather per rollout, serial) over RCCL and over the
                one-shot exchange, beside the amortised ones."""
                forms = {"serial_gather_per_rollout": run_serial_p(1)}
                if xg is not None:
                    forms["ipc_one_shot_per_rollout"] = run_ipc
                if G > 1:
                    forms[f"serial_gather_per_{G}_rollouts"] = run_serial_p(G)
                    forms[f"overlap_gather_per_{G}_rollouts"] = run_overlap
                return {k: min(trial(f) for _ in range(3)) / (4 * G) * 1e3 for k, f in forms.items()}
    else:
        G = 1

        def run():
            R.step()
            if dist:
                rd.gather_episode(R.env.ep)

    for _ in range(-(-args.warmup // G)):
        run()

    def timed_trial():
        """EXACTLY --steps rollouts between a barrier + synchronize on both sides; the max over
        ranks of the wall time (identical on every rank, so every rank takes the same number of
        trials)."""
        if dist:
            tdist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps // G):
            run()
        torch.cuda.synchronize()  # every stream: the last set's gather is inside the timed region
        if dist:
            tdist.barrier()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], dtype=torch.float64, device=device)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # the --steps loop repeated until >= 1000 rollouts and >= 0.2 s were timed; the median
    # trial is reported (a 20-step trial is ~0.5 ms: one trial alone is noise)
    trials = [timed_trial()]
    while len(trials) < 200 and (len(trials) * args.steps < 1000 or sum(trials) < 0.2):
        trials.append(timed_trial())
    elapsed = float(np.median(trials))
    total_steps = steps_per_rollout * args.steps
    if dist:
        c = torch.tensor([total_steps], dtype=torch.float64, device=device)
        tdist.all_reduce(c)
        total_steps = int(c.item())
    # every replayed rollout wrote a full record (deterministic: all arenas identical), and at
    # N > 1 EVERY rank's row of each gathered set equals the digest that rank broadcast of its
    # own set (this rank's row also byte for byte)
    exchange_ok = None
    gathered_info = None
    if graph is not None:
        exchange_ok = all(torch.equal(e.arena, eps[0].arena) for e in eps)
        if dist and transport == "ipc":
            r = tdist.get_rank()
            torch.cuda.synchronize()
            for e in (xg.epoch - 1, xg.epoch):  # the two slots: the last two rollouts' gathers
                exchange_ok = check_gathered(eps[0].arena, xg.slot(e).contiguous().view(-1), W, r,
                                             distinct=True) and exchange_ok
            xg_err = xg.error()
            exchange_ok = exchange_ok and xg_err == 0
            gathered_info = {"ranks": W, "bytes_per_rank_per_gather": int(arena_bytes),
                             "bytes_per_gather": int(W * arena_bytes), "rollouts_per_gather": 1,
                             "transport": "ipc", "exchanges": xg.epoch, "err_bits": xg_err,
                             "check": "every rank's row of the last two gathered slots == the i64 digest that "
                                      "rank all-gathered of its own arena; own row byte for byte"}
        elif dist:
            r = tdist.get_rank()
            p_run = G if exchange_mode == "overlap" else P
            for h in (0, 1):
                for k in range(G // p_run):
                    exchange_ok = check_gathered(chunk(h, p_run, k), outs[p_run][h][k], W, r,
                                                 distinct=True) and exchange_ok
            gathered_info = {"ranks": W, "bytes_per_rank_per_gather": int(p_run * arena_bytes),
                             "bytes_per_gather": int(W * p_run * arena_bytes), "rollouts_per_gather": p_run,
                             "transport": "rccl",
                             "check": "every rank's row of every gathered chunk == the i64 digest that rank "
                                      "all-gathered of its own chunk; own row byte for byte"}
        ok_t = torch.tensor([1 if exchange_ok else 0], dtype=torch.int32, device=device)
        if dist:
            tdist.all_reduce(ok_t, op=tdist.ReduceOp.MIN)
        exchange_ok = bool(ok_t.item())
        if not exchange_ok:
            raise RuntimeError("replayed rollouts / gathered arenas do not match")
        if dist:  # every placement timed beside the headline (collective: every rank)
            variants = variants_fn()

    # ---- dominant-kernel roofline: HIP events around the turn launches (eager, same stream)
    n_prof = min(args.steps, 50)
    events = [R.timed_turns() for _ in range(n_prof)]
    torch.cuda.synchronize()
    durs = np.array([a.elapsed_time(b) for a, b in events]) * 1e-3  # s per rollout's T launches
    bytes_per_rollout = float(np.sum(active_per_turn)) * BYTES_PER_ENV_TURN
    achieved = bytes_per_rollout * n_prof / float(durs.sum()) / 1e9  # GB/s
    avg_launch_us = float(durs.mean() / T_TURNS * 1e6)
    traffic = _pmc_field(PMC_GLOB, "hbm_bytes_per_launch")

    # eager (no graph) rate, for reference
    eager_steps = 20
    torch.cuda.synchronize()
    te = time.perf_counter()
    for _ in range(eager_steps):
        R.step()
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - te) / eager_steps * 1e3

    # the extras (and the CPU baselines below) run on rank 0 only: the other ranks' GPUs hold
    # identical work, and the headline above is already timed
    extras = not args.no_extras and rank == 0
    adv = advantage_leg(R, device) if extras else None
    copy_probe = hbm_copy_peak(device) if extras else None
    # frac_of_achievable's denominator: the larger of this box's probe and the guide's measured
    # float4 copy (MI355X_MICROARCH.md: 6.29 TB/s), so a slow probe never inflates the fraction
    copy_peak = max(copy_probe, GUIDE_COPY_GBS) if copy_probe else None
    toytext = toytext_legs(device) if extras else None
    api = api_leg(device) if not args.no_extras and rank == 0 else None
    text = text_leg(R, device) if not args.no_extras and rank == 0 else None
    if text is not None and api is not None:  # the caller path's text kernels (measured in api_leg)
        text["prompt"] = api.pop("prompt_kernels", None)
    if text is not None:
        attach_issue_fracs(text)
    at_scale = None
    if not args.no_extras and rank == 0:
        s_dur, s_B = scale_leg(R, device)
        s_bytes = bytes_per_rollout * (s_B // R.B)
        s_ach = s_bytes / s_dur / 1e9
        tile = s_B // R.B
        act = np.tile(np.stack([n_turns > t for t in range(T_TURNS)]), (1, tile))
        floor = layout_floor(act)
        algo_read = float(act.sum()) * 83 / T_TURNS  # 83 of the 141 B per active env-turn are reads
        pmc_read = _pmc_field(PMC_SCALE_GLOB, "read_bytes_per_launch")
        at_scale = {"envs": s_B, "avg_launch_us": s_dur / T_TURNS * 1e6, "achieved": s_ach,
                    "frac": s_ach / HBM_PEAK_GBS, "frac_of_achievable": (s_ach / copy_peak) if copy_peak else None,
                    "algorithmic_MB_per_launch": s_bytes / T_TURNS / 1e6,
                    "cache": "out of the 256 MiB Infinity Cache (per-launch footprint ~420 MB): HBM-bound",
                    "traffic": _pmc_field(PMC_SCALE_GLOB, "hbm_bytes_per_launch"),
                    "reads": {"algorithmic_MB_per_launch": algo_read / 1e6,
                              "layout_floor_MB_per_launch": {f"{k}B_lines": v for k, v in floor.items()},
                              "pmc_MB_per_launch": pmc_read / 1e6 if pmc_read else None,
                              "note": "layout floor: every env's 21 B of flags / scalars / actions plus the grid "
                                      "lines an acting env's 36-B rows touch (done envs interleaved with acting "
                                      "ones in the caller's SoA), bench.layout_floor"},
                    "note": "same kernel and workload per env, batch tiled 512x"}

    if rank == 0:
        cpu = cpu_par = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(R)
            except Exception as ex:  # the baseline must never break the bench line
                cpu = {"value": None, "unit": "env-steps/s", "cores": 1, "kind": "port", "sample": f"failed: {ex}"}
            try:
                cpu_par = cpu_baseline_parallel(R)
            except Exception as ex:
                cpu_par = {"value": None, "sample": f"failed: {ex}"}
            if adv is not None:
                try:
                    adv["cpu_baseline"] = cpu_gae_baseline(R)
                    adv["speedup_vs_cpu_1t"] = adv["tokens_per_s"] / adv["cpu_baseline"]["tokens_per_s_1t"]
                except Exception as ex:
                    adv["cpu_baseline"] = {"value": None, "sample": f"failed: {ex}"}
        value = total_steps / elapsed
        assert world == args.gpus, (world, args.gpus)
        line = {
            "metric": "env-steps/sec (whole node), Sokoban 6x6, 8192 envs x 5 turns",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "timing": {"trials": len(trials), "rollouts_timed": len(trials) * args.steps,
                       "seconds_timed": float(np.sum(trials)), "statistic": "median trial",
                       "ms_per_step_min_med_max": [min(trials) / args.steps * 1e3, elapsed / args.steps * 1e3,
                                                   max(trials) / args.steps * 1e3]},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (fixed-seed actions; rooms generated with the reference's exact RNG streams)",
            "config": {"workload": f"Sokoban 6x6 1-box, {B_PER_GPU} envs/GPU x {T_TURNS} turns, K={K_ACTIONS}, "
                                   f"cap {MAX_ACTIONS}, groups of {GROUP}; rollout phase (reset excluded)",
                       "envs_per_gpu": B_PER_GPU, "env_steps_per_rollout_rank0": steps_per_rollout,
                       "graph": graph is not None, "rollouts_per_replay": G, "parallelism": f"env-sharded x{world}",
                       "board_cache": R.boards,
                       "exchange_mode": exchange_mode if dist else None,
                       "exchange_transport": transport, "exchange_transport_note": xg_note,
                       "rollouts_per_gather": (G if exchange_mode == "overlap" else P) if dist else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": _pmc_source(PMC_GLOB),
                         "achievable_peak": copy_peak,
                         "achievable_peak_probe": copy_probe, "achievable_peak_guide": GUIDE_COPY_GBS,
                         "achievable_peak_rule": "max(probe on this box, guide's float4 copy)",
                         "frac_of_achievable": (achieved / copy_peak) if copy_peak else None,
                         "kernel": "rmi_sokoban_step_turn", "avg_launch_us": avg_launch_us,
                         "bytes_per_env_turn": BYTES_PER_ENV_TURN, "active_envs_per_turn": active_per_turn,
                         "timed_region": {
                             "avg_launch_us": elapsed / args.steps / T_TURNS * 1e6,
                             "achieved": bytes_per_rollout * args.steps / elapsed / 1e9,
                             "frac": bytes_per_rollout * args.steps / elapsed / 1e9 / HBM_PEAK_GBS,
                             "note": "the same bytes over the timed region itself (graph replays of the fused "
                                     "first / plain / last-turn launches, boundaries included); `achieved` "
                                     "above brackets 5 plain launches with events, as rocprof times them"},
                         "at_scale": at_scale},
            "cpu_baseline": cpu,
            "cpu_baseline_parallel": cpu_par,
            "advantage": adv,
            "toytext": toytext,
            "api_variant": api,
            "text_api": text,
            "exchange": exchange_label(exchange_mode, P, G, args.exchange, graph is not None, transport) if dist else None,
            "exchange_variants_ms_per_rollout": variants,
            "records_checked": exchange_ok,
            "gathered": gathered_info,
            "eager_ms_per_step": eager_ms,
            "speedup_vs_cpu_baseline": (value / cpu["value"]) if cpu and cpu.get("value") else None,
        }
        print(json.dumps(line), flush=True)
    if dist:
        if xg is not None:
            torch.cuda.synchronize()
            tdist.barrier()  # no rank unmaps a region a peer may still store into
            xg.close()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
