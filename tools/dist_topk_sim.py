"""CPU simulation (oracle env, one C5-shaped env: 16 agents, 512x512, lidar
21 beams R=10) of how many full distance transforms two rules need:
  witness rule (built): a map is transformed when a newly covered cell comes
    closer than M to the witness;
  top-K cache: the transform also records every cell with
    d >= M - T (at most K); a listed map takes the largest current d of its
    cached cells while that stays >= M0 - T, else it is transformed again.
    python tools/dist_topk_sim.py T K STEPS     e.g. 8 128 40
"""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
from oracle.cpu_ref import DecGridRLRef, l1_distance_to_covered
T, K = int(sys.argv[1]), int(sys.argv[2])
rs = np.random.RandomState(3)
grid = rs.choice([1.0, -1.0], size=(512, 512), p=[0.9, 0.1])
cfg = dict(numrobot=16, maxsteps=2000, train_maxsteps=2000, test_maxsteps=2000, collision_penalty=5,
           terminal_reward=30, done_thresh=1, done_incr=0, egoradius=2, mini_map_rad=0, comm_radius=0,
           allow_comm=0, map_sharing=0, single_square_tool=0, dijkstra_input=0, dist_reward=0,
           sensor_type='lidar', sensor_config={"num_lasers": 21, "range": 10})
np.random.seed(0)
env = DecGridRLRef([grid], cfg)
env.reset(False, None)
N = 16
state = []  # per agent: M, witness, cache (cells, M0)
def transform(i):
    d = l1_distance_to_covered(env._free_pad[i])
    M = int(d.max())
    cells = np.argwhere(d >= M - T)
    return d, M, cells
wit_tx = top_tx = 0; over = 0
info = []
for i in range(N):
    d, M, cells = transform(i)
    w = tuple(np.argwhere(d == M)[0])
    info.append(dict(M=M, w=w, M0=M, cache=cells if len(cells) <= K else None))
steps = int(sys.argv[3])
for t in range(steps):
    prev = [env._free_pad[i].copy() for i in range(N)]
    env.step(rs.randint(0, 4, size=N))
    for i in range(N):
        new = np.argwhere((env._free_pad[i] > 0) & (prev[i] == 0))
        st = info[i]
        d = l1_distance_to_covered(env._free_pad[i])
        Mtrue = int(d.max())
        # witness rule
        wd = np.abs(new - np.array(st['w'])).sum(1).min() if len(new) else 10**9
        wit_list = wd < st['M']
        # top-K rule: cached cells' current d (exact)
        ok = False
        if st['cache'] is not None:
            cd = d[tuple(st['cache'].T)]
            if cd.max() >= st['M0'] - T:
                ok = True
                assert cd.max() == Mtrue, (cd.max(), Mtrue)
        if wit_list:
            wit_tx += 1
            if not ok:
                top_tx += 1
                cells = np.argwhere(d >= Mtrue - T)
                st['cache'] = cells if len(cells) <= K else None
                st['M0'] = Mtrue
                if st['cache'] is None: over += 1
            st['M'] = Mtrue
            st['w'] = tuple(np.argwhere(d == Mtrue)[0])
print(f"T={T} K={K} steps={steps}: witness-rule transforms {wit_tx}, top-K transforms {top_tx}, overflows {over} of {steps*N} map-steps")
