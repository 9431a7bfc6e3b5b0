"""DecGridRL: drop-in facade of the reference environment, stepped on the GPU.

Same constructor, methods, attributes and return types as
``Environments/dec_grid_rl.py:DecGridRL`` (ExistentialRobotics/MARL-Coverage),
so the reference's controllers and episode loop (``Utils/utils.py``) run
unchanged.  Every step is one launch of the HIP env kernel (batch of 1); the
host keeps only what the reference's callers read back.

Randomness is the reference's: ``reset`` draws the grid index and the robot
start cells from NumPy's global RNG with the same call sequence
(dec_grid_rl.py:466-502), then injects the cells into the device env, so a
seeded run reproduces the reference's trajectory bit for bit.

Differences (deliberate supersets): per-agent action arrays/lists are accepted
for any ``numrobot`` (the reference raises ValueError on them for N > 1,
SURVEY §8(a) a1); ``render`` returns the composed RGB frame without pygame.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .batch_env import BatchCoverageEnv, pad_grid
from .sensors import make_sensor
from .tiles import tiles_to_cells

_DIRS = (0, 1, 2, 3)


def decode_action(action, numrobot):
    """Reference action decoding (dec_grid_rl.py:104-117) -> uint8 codes [N].

    Returns None for the sentinel (``action == None or action == -1``)."""
    if action is None:
        return None
    if isinstance(action, (list, tuple)):
        action = np.asarray(action)
    if isinstance(action, np.ndarray):
        flat = action.reshape(-1)
        if flat.size == 1 and flat[0] == -1:
            return None
        ulis = flat
    else:
        try:
            if action == -1:
                return None
        except Exception:
            pass
        ulis = np.zeros((numrobot,))
        for i in range(numrobot):
            ulis[i] = action % 4
            action = action // 4
    codes = np.full(numrobot, _lib.ACT_NOOP, dtype=np.uint8)
    for i in range(min(numrobot, len(ulis))):
        u = ulis[i]
        for d in _DIRS:
            if u == d:
                codes[i] = d
                break
    return codes


class DecGridRL:
    """GPU-backed ``DecGridRL(train_set, env_config, use_graph, test_set)``."""

    def __init__(self, train_set, env_config, use_graph=False, test_set=None, device="cuda"):
        import torch

        self._torch = torch
        self._train_gridlis = train_set
        self._test_gridlis = test_set
        c = env_config
        self._env_config = dict(env_config)
        self._numrobot = c["numrobot"]
        self._maxsteps = c["maxsteps"]
        self._collision_penalty = c["collision_penalty"]
        self._dt = c["done_thresh"]           # host mirror of the device value
        self._done_incr = c["done_incr"]
        self._terminal_reward = c["terminal_reward"]
        self._dist_r = c["dist_reward"]
        self._train_maxsteps = c["train_maxsteps"]
        self._test_maxsteps = c["test_maxsteps"]
        self._egoradius = c["egoradius"]
        self._mini_map_rad = c["mini_map_rad"]
        self._comm_radius = c["comm_radius"]
        self._allow_comm = c["allow_comm"]
        self._map_sharing = c["map_sharing"]
        self._use_graph = use_graph
        self._single_square_tool = c["single_square_tool"]
        self._dijkstra_input = c["dijkstra_input"]
        self._sensor = make_sensor(c)
        self._pad = max(self._egoradius, self._mini_map_rad)
        self._device = torch.device(device)
        self._envs = {}          # padded shape -> (BatchCoverageEnv, [pool grid ids])
        self._pool_index = {}    # id(caller's grid object) -> (padded shape, pool index)
        self._env = None
        self.reset(False, None)
        self._obs_dim = self.get_egocentric_observations()[0].shape
        self._num_actions = 4

    # ---- device env per padded grid shape ----------------------------------
    def _device_env(self, raw):
        """The pool env of ``raw``'s padded shape and ``raw``'s index in it.
        The pool is keyed on the caller's own grid objects (the train/test
        list entries): lists of lists are accepted like the reference's
        ``np.pad`` accepts them, and converting them per reset would make a
        new object every time."""
        shape = np.asarray(raw).shape
        padded_shape = (shape[0] + 2, shape[1] + 2)
        hit = self._pool_index.get(id(raw))
        if (padded_shape in self._envs and hit is not None and hit[0] == padded_shape
                and self._envs[padded_shape][1][hit[1]] is raw):
            return self._envs[padded_shape][0], hit[1]
        # a miss: the pool of this shape is rebuilt from the CURRENT train /
        # test lists (entries the caller replaced drop out, so the pool does
        # not grow with every replacement), plus ``raw`` if it is in neither
        uniq, seen = [], set()
        for g in list(self._train_gridlis or []) + list(self._test_gridlis or []):
            if id(g) not in seen and np.asarray(g).shape == shape:
                seen.add(id(g))
                uniq.append(g)
        if id(raw) not in seen:
            uniq.append(raw)
        if padded_shape in self._envs:
            self._envs.pop(padded_shape)[0].close()
            if self._env is not None and self._env._h is None:
                self._env = None
        env = BatchCoverageEnv(self._env_config, 1, grids=[np.asarray(g) for g in uniq],
                               device=self._device, auto_reset=False, sensor=self._sensor,
                               want_adjacency=True)
        self._envs[padded_shape] = (env, uniq)
        # forget the evicted grids of this shape (ids of dead objects get reused)
        self._pool_index = {k: v for k, v in self._pool_index.items() if v[0] != padded_shape}
        self._pool_index.update({id(g): (padded_shape, i) for i, g in enumerate(uniq)})
        return env, self._pool_index[id(raw)][1]

    def _push_done_thresh(self, env):
        t = self._torch.tensor([float(self._dt)], dtype=self._torch.float64)
        env.set_state(_lib.FIELD_DONE_THRESH, t)

    @property
    def _done_thresh(self):
        """``_done_thresh`` persists across resets and grows by done_incr each
        time done() fires (dec_grid_rl.py:52,542); the device holds it."""
        return self._dt

    @_done_thresh.setter
    def _done_thresh(self, value):
        self._dt = value
        if getattr(self, "_env", None) is not None:
            self._push_done_thresh(self._env)

    # ---- reference API ------------------------------------------------------
    def reset(self, testing, ind):
        """``dec_grid_rl.py:449-531`` (same NumPy RNG call sequence)."""
        if testing and self._test_gridlis is not None:
            raw = self._test_gridlis[ind]
        else:
            raw = self._train_gridlis[np.random.randint(len(self._train_gridlis))]
        grid = pad_grid(raw)
        self._grid = grid
        self._gridwidth, self._gridlen = grid.shape
        self._currstep = 0
        n = self._numrobot
        xs = np.zeros(n, dtype=int)
        ys = np.zeros(n, dtype=int)
        taken = np.zeros(grid.shape, dtype=bool)
        count = 0
        while count != n:
            x = np.random.randint(self._gridwidth)
            y = np.random.randint(self._gridlen)
            if grid[x][y] >= 0 and not taken[x][y]:
                taken[x][y] = True
                xs[count], ys[count] = x, y
                count += 1
        env, idx = self._device_env(raw)
        if self._env is not env:
            self._env = env
            self._push_done_thresh(env)
        env.set_env_grids([idx])
        pos = np.stack([xs, ys], axis=1)[None].astype(np.int32)
        env.reset(positions=pos)
        self._xinds, self._yinds = xs, ys
        self._robot_pos_map = taken.astype(np.float64)
        self._numfree = int(np.count_nonzero(grid > 0))
        self._numobserved = 0
        self._refresh(reset=True)
        obs = self._obs_np
        if self._allow_comm and self._use_graph:
            return obs, self._grid, self._adjacency_matrix
        return obs, self._grid

    def step(self, action):
        """``dec_grid_rl.py:91-169``."""
        env = self._env
        codes = decode_action(action, self._numrobot)
        sentinel = codes is None
        # the action row goes through a cached pinned buffer (asynchronous
        # copy, ordered before the step on the stream)
        torch = self._torch
        ab = self.__dict__.get("_act_buf")
        if ab is None or ab[0].shape[1] != self._numrobot or ab[1].device != torch.device(env.device):
            ab = self._act_buf = (torch.empty((1, self._numrobot), dtype=torch.uint8, pin_memory=True),
                                  torch.empty((1, self._numrobot), dtype=torch.uint8, device=env.device))
        host, dev = ab
        h = host.numpy()
        h[0] = _lib.ACT_SENTINEL if sentinel else codes
        dev.copy_(host, non_blocking=True)
        env.step(dev)
        self._refresh(reset=False)
        if sentinel:
            reward, done = 0, True
        else:
            reward = np.float64(self._reward_dev)
            done = bool(self._done_dev)
        obs = self._obs_np
        if self._allow_comm and self._use_graph:
            return [obs, self._adjacency_matrix], reward, done
        return obs, reward, done

    def _fetch(self, tensors):
        """Device tensors -> NumPy arrays with ONE stream synchronization: each
        is copied asynchronously into a cached pinned host buffer on the env's
        stream (ordered after the step), then the stream is synchronized once
        (the per-field ``.cpu()`` / ``.item()`` calls were one blocking copy
        each: 160 -> 122 us per facade step, tools/facade_probe.py)."""
        torch = self._torch
        cache = self.__dict__.setdefault("_pinned", {})
        out = []
        for i, t in enumerate(tensors):
            key = (i, tuple(t.shape), t.dtype)
            h = cache.get(key)
            if h is None:
                h = cache[key] = torch.empty(t.shape, dtype=t.dtype, pin_memory=t.is_cuda)
            h.copy_(t, non_blocking=t.is_cuda)
            out.append(h)
        if any(t.is_cuda for t in tensors):
            torch.cuda.current_stream(self._env.device).synchronize()
        return [h.numpy() for h in out]

    def _refresh(self, reset):
        env = self._env
        bufs = self.__dict__.get("_state_bufs")
        if bufs is None or bufs[0] is not env:
            torch = self._torch
            bufs = self._state_bufs = (env, {f: torch.empty(env.field_shape(f), dtype=getattr(torch, d),
                                                            device=env.device)
                                             for f, d in ((_lib.FIELD_POS, "int32"),
                                                          (_lib.FIELD_CURRSTEP, "int32"),
                                                          (_lib.FIELD_DONE_THRESH, "float64"))})
        sb = bufs[1]
        pieces = [env.obs[0], env.get_state(_lib.FIELD_POS, out=sb[_lib.FIELD_POS])[0],
                  env.get_state(_lib.FIELD_CURRSTEP, out=sb[_lib.FIELD_CURRSTEP])[:1],
                  env.get_state(_lib.FIELD_DONE_THRESH, out=sb[_lib.FIELD_DONE_THRESH])[:1],
                  env.reward[:1], env.done[:1]]
        dist = env.dist_obs is not None and not self._dijkstra_input
        if dist:
            pieces.append(env.dist_obs[0])
        if env.minimap_obs is not None:
            pieces.append(env.minimap_obs[0])
        if env.adj is not None:
            pieces.append(env.adj[0])
        got = self._fetch(pieces)
        obs, pos, cs, dt, rew, dn = got[:6]
        rest = got[6:]
        self._obs_np = obs.astype(np.float64)
        if dist:
            # float distance layer (the dijkstra path overwrites it, :354-358)
            self._obs_np[:, 3] = rest.pop(0).astype(np.float64)
        if env.minimap_obs is not None:  # overwrites layers 3 and 4 (:365-370)
            self._obs_np[:, 3:5] = rest.pop(0)
        self._xinds = pos[:, 0].astype(int)
        self._yinds = pos[:, 1].astype(int)
        if env.adj is not None:
            self._adjacency_matrix = rest.pop(0).astype(np.float64)
        self._currstep = int(cs[0])
        if float(dt[0]) != float(self._dt):
            self._dt = float(dt[0])
        if not reset:
            self._reward_dev = float(rew[0])
            self._done_dev = int(dn[0])
        rp = np.zeros(self._grid.shape)
        rp[self._xinds, self._yinds] = 1
        self._robot_pos_map = rp

    def get_egocentric_observations(self):
        return self._obs_np.copy()

    def percent_covered(self):
        """``dec_grid_rl.py:548-552``."""
        fc = int(self._env.get_state(_lib.FIELD_FREE_COUNT)[0].item())
        return fc / self._numfree

    def done(self):
        """``dec_grid_rl.py:533-546`` (without the print)."""
        if min(self._done_thresh, 1) <= self.percent_covered():
            self._done_thresh += self._done_incr
            self._push_done_thresh(self._env)
            return True
        if self._currstep == self._maxsteps:
            return True
        return False

    def isInBounds(self, x, y):
        return x >= 0 and x < self._gridwidth and y >= 0 and y < self._gridlen

    def isOccupied(self, x, y):
        return self._grid[x][y] < 0 or self._robot_pos_map[x][y] == 1

    # ---- reference state arrays, materialised from the device on demand ----
    def _unpack(self, tiles):
        return tiles_to_cells(tiles.cpu().numpy(), self._gridwidth, self._gridlen).astype(np.float64)

    def _padded(self, inner):
        p = self._pad
        pad = [(0, 0)] * (inner.ndim - 2) + [(p, p), (p, p)]
        return np.pad(inner, pad)

    @property
    def _free_pad(self):
        return self._padded(self._unpack(self._env.get_state(_lib.FIELD_FREE)[0]))

    @property
    def _obst_pad(self):
        return self._padded(self._unpack(self._env.get_state(_lib.FIELD_OBST)[0]))

    @property
    def _visited(self):
        return self._unpack(self._env.get_state(_lib.FIELD_VISITED)[0])

    @property
    def _observed_obstacles(self):
        return np.clip(self._unpack(self._env.get_state(_lib.FIELD_OBST)[0]).sum(axis=0), 0, 1)

    @property
    def _robot_pad(self):
        moved = int(self._env.get_state(_lib.FIELD_MOVED)[0].item()) & ((1 << 64) - 1)
        rp = np.zeros((self._gridwidth + 2 * self._pad, self._gridlen + 2 * self._pad))
        for i in range(self._numrobot):
            if (moved >> i) & 1:
                rp[self._xinds[i] + self._pad, self._yinds[i] + self._pad] = 1
        return rp

    def render(self):
        """RGB frame of ``dec_grid_rl.py:561-580`` (no pygame / cv2 scaling)."""
        image = np.zeros((self._gridwidth, self._gridlen, 3))
        ob = self._observed_obstacles
        image += np.stack([200 * ob, 0 * ob, 255 * ob], -1)
        vis = self._visited
        image += np.stack([0 * vis, 225 * vis, 255 * vis], -1)
        rp = self._robot_pos_map
        image += np.stack([255 * rp, 0 * rp, 0 * rp], -1)
        return image

    def snapshot(self):
        """Comparable state (same keys as the oracle's snapshot())."""
        return {
            "xinds": self._xinds.copy(), "yinds": self._yinds.copy(),
            "free_pad": (self._free_pad > 0).astype(np.uint8),
            "obst_pad": (self._obst_pad > 0).astype(np.uint8),
            "robot_pad": (self._robot_pad > 0).astype(np.uint8),
            "visited": (self._visited > 0).astype(np.uint8),
            "adjacency": self._adjacency_matrix.copy(),
            "currstep": int(self._currstep),
            "done_thresh": float(self._dt),
        }
