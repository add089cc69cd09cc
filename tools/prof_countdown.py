import sys, time, numpy as np, torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from ragen_amd import ops, synthetic
from ragen_amd.env import CountdownBatch
from ragen_amd.env.configs import CountdownEnvConfig
from ragen_amd.env.countdown import synthetic_instances
dev = torch.device("cuda", 0)
B, K = 16384, 1
inst = synthetic_instances(1024, 7)
cd = CountdownBatch(CountdownEnvConfig(data=inst), B, 1, K, dev)
cd.reset(synthetic.env_seeds(B))
ONLY = sys.argv[1] if len(sys.argv) > 1 else None


def run(answers, label):
    if ONLY and label != ONLY:
        return
    lists = [[a] if a is not None else [] for a in answers]
    buf, lens = cd.encode_answers(lists)
    bt, lt = torch.from_numpy(buf).to(dev), torch.from_numpy(lens).to(dev)
    n = torch.from_numpy(np.array([len(x) for x in lists], np.uint8)).to(dev)
    z = torch.zeros(B, K, dtype=torch.int8, device=dev)
    t = ops.turn_struct(0, z, n, None, 1, -0.1)
    ones = torch.ones(B, dtype=torch.uint8, device=dev)
    tb = ops.turn_struct(0, z, n, ones, 200, -0.1)  # every env steps again: back-to-back launches
    st = cd.struct()
    for _ in range(3):
        cd.ep.arena.zero_(); ops.countdown_step_turn(st, cd.ep, t, bt, lt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot = 0
    for _ in range(20):
        cd.ep.arena.zero_()
        e0.record(); ops.countdown_step_turn(st, cd.ep, t, bt, lt); e1.record(); torch.cuda.synchronize()
        tot += e0.elapsed_time(e1)
    torch.cuda._sleep(1_000_000)
    e0.record()
    for _ in range(50):
        ops.countdown_step_turn(st, cd.ep, tb, bt, lt)
    e1.record()
    torch.cuda.synchronize()
    print(label, round(tot / 20 * 1000, 1), "us single,", round(e0.elapsed_time(e1) * 1000 / 50, 1), "us back-to-back")
insts = [inst[int(i)] for i in cd.index]
run([None] * B, "empty")
run(["1"] * B, "one digit")
run([" + ".join(str(x) for x in i["nums"]) for i in insts], "sum of nums")
run(synthetic.countdown_answers(insts, 1, p_empty=0.0)[0], "synthetic mix")
run(["(" * 10 + "1" + ")" * 10] * B, "nested")
run([None] * B, "empty")
mix = synthetic.countdown_answers(insts, 1, p_empty=0.0)[0]
run([a if i % 2 == 0 else None for i, a in enumerate(mix)], "mix half")
run([a if i % 16 == 0 else None for i, a in enumerate(mix)], "mix 1/16")
run([a if i % 1024 == 0 else None for i, a in enumerate(mix)], "mix 1/1024")
