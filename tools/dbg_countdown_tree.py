import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import oracle
from ragen_amd import ops
from ragen_amd.env import CountdownBatch
from ragen_amd.env.configs import CountdownEnvConfig
src = open('tests/test_gpu_parity.py').read()
ns = {}
exec(src[src.index('def _tree_answers'):src.index('def test_countdown_reward_tree_shapes')], {'np': np}, ns)
exprs, data = ns['_tree_answers'](20000, 11)
ns2 = {}
exec(src[src.index('def _past_int64'):src.index('def test_countdown_reward_tree_shapes')], ns2)
dev = torch.device('cuda', 0)
n = len(exprs)
env = CountdownBatch(CountdownEnvConfig(data=data), n, 1, 1, dev, max_answer_bytes=64, max_nums=8)
env.reset(np.arange(n, dtype=np.int64))
buf, lens = env.encode_answers([[e] for e in exprs])
r, fl, err = ops.countdown_reward(env.struct(), torch.from_numpy(buf[:, 0].copy()).to(dev), torch.from_numpy(lens[:, 0].copy()).to(dev))
r, fl, err = r.cpu().numpy(), fl.cpu().numpy(), err.cpu().numpy()
want = np.array([oracle.countdown_reward(e, d['nums'], d['target']) for e, d in zip(exprs, data)])
big = np.array([ns2['_past_int64'](e) for e in exprs])
for i in np.nonzero((r != want) | (err.astype(bool) & ~big))[0]:
    try:
        v = eval(exprs[i], {"__builtins__": None}, {})
    except Exception as ex:
        v = repr(ex)
    print(repr(exprs[i]), 'big', big[i], data[i], 'got', r[i], 'want', want[i], 'err', err[i], 'pyval', v)
