"""SuperGridRL on the GPU: the centralized, fully observed env variant
(``Environments/super_grid_rl.py:18-463``).

``BatchSuperGridEnv`` steps B envs per launch through the ``mc_sg_*`` C ABI
(include/marlcov.h, csrc/mc_super.hip); PyTorch only provides device memory
and the stream.  ``SuperGridRL`` is the drop-in facade with the reference's
constructor, methods, attributes and return types, driving a one-env batch
and reproducing the reference's NumPy RNG call sequence for resets.

There is no CPU fallback: without libmarlcov.so the classes raise.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .batch_env import grid_to_int8

_SG_DTYPES = {
    _lib.SG_FIELD_POS: "int32", _lib.SG_FIELD_COVERED: "int64", _lib.SG_FIELD_OBST: "int64",
    _lib.SG_FIELD_COV_COUNT: "int32", _lib.SG_FIELD_CURRSTEP: "int32",
    _lib.SG_FIELD_DONE_THRESH: "float64", _lib.SG_FIELD_A_PREV: "int32",
    _lib.SG_FIELD_ENV_GRID: "int32", _lib.SG_FIELD_EPISODE: "int32", _lib.SG_FIELD_NUMPOS: "int32",
    _lib.SG_FIELD_GRID_NEG: "int64", _lib.SG_FIELD_GRID_POS: "int64",
    _lib.SG_FIELD_EP_PC: "float64", _lib.SG_FIELD_EP_LEN: "int32",
}


def unpack_rows(words, length):
    """uint64 row bitboards [..., W, RW] -> uint8 cells [..., W, L]."""
    w = np.ascontiguousarray(np.asarray(words).view(np.uint64))
    bits = np.unpackbits(w.view(np.uint8), axis=-1, bitorder="little")
    return bits.reshape(w.shape[:-1] + (w.shape[-1] * 64,))[..., :length]


def pack_rows(cells):
    """uint8/bool cells [..., W, L] -> uint64 row bitboards [..., W, ceil(L/64)]."""
    c = np.asarray(cells).astype(bool)
    L = c.shape[-1]
    RW = (L + 63) // 64
    padded = np.zeros(c.shape[:-1] + (RW * 64,), dtype=bool)
    padded[..., :L] = c
    by = np.packbits(padded, axis=-1, bitorder="little")
    return np.ascontiguousarray(by).view(np.uint64)


class BatchSuperGridEnv:
    """``num_envs`` independent SuperGridRL envs on one HIP device.

    ``grids``: UNPADDED pool grids of one shape (values in {-1, 0, 1}); or
    ``gen=dict(width=, length=, prob_obst=, seed=, num_grids=)``.

    State buffers (library-maintained, overwritten by every call):
    ``planes`` uint8 [B, P+2, W, L] (P robot-position layers — N, or 1 with
    ``use_scanning`` —, observed obstacles, _free) and ``dist`` float32
    [B, W, L] (the distance-map layer).  ``step`` returns
    ``((planes, dist), reward float64 [B], done uint8 [B])``.
    ``maxsteps`` > 0 adds the episode cut of ``Utils/utils.py:25-28``.
    """

    def __init__(self, env_config, num_envs, grids=None, *, gen=None, device="cuda", seed=0,
                 auto_reset=True, maxsteps=0, reset_grid_mode="keep", env_grid=None, env_offset=0,
                 grid_offset=None):
        import torch

        self._torch = torch
        self.lib = _lib.load()
        self.config = dict(env_config)
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("BatchSuperGridEnv needs a HIP device (torch 'cuda' device)")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.num_envs = int(num_envs)
        self.num_agents = int(self.config["numrobot"])
        if (grids is None) == (gen is None):
            raise ValueError("give exactly one of grids= or gen=")
        if grids is not None:
            arrs = [np.asarray(g, dtype=np.float64) for g in grids]
            shapes = {a.shape for a in arrs}
            if len(shapes) != 1:
                raise ValueError(f"all pool grids must share one shape, got {sorted(shapes)}")
            self.width, self.length = arrs[0].shape
            self.num_grids = len(arrs)
        else:
            self.width, self.length = int(gen["width"]), int(gen["length"])
            self.num_grids = int(gen.get("num_grids", self.num_envs))

        c = _lib.McSgConfig()
        c.num_envs, c.num_agents = self.num_envs, self.num_agents
        c.width, c.length, c.num_grids = self.width, self.length, self.num_grids
        c.senseradius = int(self.config["senseradius"])
        c.collision_penalty = float(self.config["collision_penalty"])
        c.free_penalty = float(self.config["free_penalty"])
        c.terminal_reward = float(self.config["terminal_reward"])
        c.done_thresh = float(self.config["done_thresh"])
        c.done_incr = float(self.config["done_incr"])
        c.dist_reward = int(bool(self.config["dist_reward"]))
        c.use_scanning = int(bool(self.config["use_scanning"]))
        c.maxsteps = int(maxsteps)
        c.auto_reset = int(bool(auto_reset))
        c.reset_grid_mode = {"keep": 0, "random": 1}[reset_grid_mode]
        c.seed = int(seed) & (2 ** 64 - 1)
        c.env_offset = int(env_offset)  # global ids (BatchCoverageEnv)
        c.grid_offset = int(env_offset if grid_offset is None else grid_offset)
        self._cfg = c
        h = ctypes.c_void_p()
        _lib.check(self.lib.mc_sg_create(ctypes.byref(c), dev.index, ctypes.byref(h)), "mc_sg_create")
        self._h = h
        lay = _lib.McSgLayout()
        _lib.check(self.lib.mc_sg_query(self._h, ctypes.byref(lay)), "mc_sg_query")
        self.layout = lay
        self.pos_layers = lay.pos_layers
        self.row_words = lay.row_words

        if grids is not None:
            self.set_grids(arrs)
        else:
            _lib.check(self.lib.mc_sg_generate_grids(self._h, int(gen.get("seed", 0)),
                                                     float(gen["prob_obst"]), self._stream()),
                       "mc_sg_generate_grids")
        if env_grid is not None:
            self.set_env_grids(env_grid)
        B, W, L = self.num_envs, self.width, self.length
        self.planes = torch.zeros((B, lay.obs_layers, W, L), dtype=torch.uint8, device=dev)
        self.dist = torch.zeros((B, W, L), dtype=torch.float32, device=dev)
        _lib.check(self.lib.mc_sg_set_obs(self._h, self.planes.data_ptr(), self.dist.data_ptr()),
                   "mc_sg_set_obs")
        self.reward = torch.zeros(B, dtype=torch.float64, device=dev)
        self.done = torch.zeros(B, dtype=torch.uint8, device=dev)

    def _stream(self):
        return ctypes.c_void_p(self._torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mc_sg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_grids(self, grids):
        host = np.stack([grid_to_int8(g) for g in grids])
        if host.shape != (self.num_grids, self.width, self.length):
            raise ValueError("grid pool shape differs from the handle's")
        d = self._torch.from_numpy(host).to(self.device)
        _lib.check(self.lib.mc_sg_set_grids(self._h, d.data_ptr(), self.num_grids, self._stream()),
                   "mc_sg_set_grids")

    def set_env_grids(self, env_grid):
        t = self._torch.as_tensor(np.asarray(env_grid, dtype=np.int32), device=self.device)
        if t.numel() != self.num_envs or int(t.min()) < 0 or int(t.max()) >= self.num_grids:
            raise ValueError("env_grid must hold num_envs indices into the grid pool")
        _lib.check(self.lib.mc_sg_set_env_grids(self._h, t.data_ptr(), self._stream()), "mc_sg_set_env_grids")

    def reset(self, env_mask=None, positions=None):
        """Reset the envs in ``env_mask`` (None = all); ``positions`` int32
        [B, N, 2] injects start cells.  Returns ``(planes, dist)``."""
        torch = self._torch
        m = None if env_mask is None else torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
        p = None
        if positions is not None:
            p = torch.as_tensor(positions, device=self.device).to(torch.int32).contiguous()
            if tuple(p.shape) != (self.num_envs, self.num_agents, 2):
                raise ValueError("positions must be [num_envs, numrobot, 2]")
        _lib.check(self.lib.mc_sg_reset(self._h, None if m is None else m.data_ptr(),
                                        None if p is None else p.data_ptr(), self._stream()), "mc_sg_reset")
        return self.planes, self.dist

    def step(self, actions, quot=None):
        """``actions`` uint8 [B, N]: the base-4 digits of each joint action
        (slot 0 first; 255 in slot 0 = sentinel).  ``quot`` int32 [B]
        (optional): ``action // 4**N``, what motion_penalty sees."""
        torch = self._torch
        a = actions
        if not (isinstance(a, torch.Tensor) and a.dtype == torch.uint8 and a.device == self.device
                and a.is_contiguous()):
            a = torch.as_tensor(a, device=self.device).to(torch.uint8).contiguous()
        if tuple(a.shape) != (self.num_envs, self.num_agents):
            raise ValueError(f"actions must be [{self.num_envs}, {self.num_agents}] uint8")
        q = None
        if quot is not None:
            q = torch.as_tensor(quot, device=self.device).to(torch.int32).contiguous()
        _lib.check(self.lib.mc_sg_step(self._h, a.data_ptr(), None if q is None else q.data_ptr(),
                                       self.reward.data_ptr(), self.done.data_ptr(), self._stream()),
                   "mc_sg_step")
        return (self.planes, self.dist), self.reward, self.done

    def step_raw(self, actions_ptr: int, reward_ptr: int, done_ptr: int, stream: int):
        """Zero-overhead launch for benchmarks."""
        return self.lib.mc_sg_step(self._h, actions_ptr, None, reward_ptr, done_ptr, stream)

    def field_shape(self, field):
        B, N, G, W, RW = self.num_envs, self.num_agents, self.num_grids, self.width, self.row_words
        return {
            _lib.SG_FIELD_POS: (B, N, 2), _lib.SG_FIELD_COVERED: (B, W, RW), _lib.SG_FIELD_OBST: (B, W, RW),
            _lib.SG_FIELD_COV_COUNT: (B,), _lib.SG_FIELD_CURRSTEP: (B,), _lib.SG_FIELD_DONE_THRESH: (B,),
            _lib.SG_FIELD_A_PREV: (B,), _lib.SG_FIELD_ENV_GRID: (B,), _lib.SG_FIELD_EPISODE: (B,),
            _lib.SG_FIELD_NUMPOS: (G,), _lib.SG_FIELD_GRID_NEG: (G, W, RW), _lib.SG_FIELD_GRID_POS: (G, W, RW),
            _lib.SG_FIELD_EP_PC: (B,), _lib.SG_FIELD_EP_LEN: (B,),
        }[field]

    def get_state(self, field):
        torch = self._torch
        t = torch.empty(self.field_shape(field), dtype=getattr(torch, _SG_DTYPES[field]), device=self.device)
        _lib.check(self.lib.mc_sg_get_state(self._h, field, t.data_ptr(), t.numel() * t.element_size(),
                                            self._stream()), "mc_sg_get_state")
        return t

    def set_state(self, field, tensor):
        torch = self._torch
        t = tensor.to(self.device).to(getattr(torch, _SG_DTYPES[field])).contiguous()
        if tuple(t.shape) != self.field_shape(field):
            raise ValueError(f"field {field} must have shape {self.field_shape(field)}")
        _lib.check(self.lib.mc_sg_set_state(self._h, field, t.data_ptr(), t.numel() * t.element_size(),
                                            self._stream()), "mc_sg_set_state")

    def percent_covered(self):
        """float64 [B]: count_nonzero(_free < 1) / count_nonzero(grid > 0) (:416-421)."""
        cc = self.get_state(_lib.SG_FIELD_COV_COUNT).to(self._torch.float64)
        npos = self.get_state(_lib.SG_FIELD_NUMPOS).to(self._torch.float64)
        eg = self.get_state(_lib.SG_FIELD_ENV_GRID).long()
        return cc / npos[eg]

    def check(self):
        _lib.check(self.lib.mc_sg_check(self._h, self._stream()), "mc_sg_check")


def decode_super_action(action, n):
    """super_grid_rl.py:88-98,203-205 -> (digit bytes [n], quotient) or None
    for the sentinel.  Ints (and 0-d tensors / NumPy integers) are split into
    base-4 digits, slot 0 least significant; the quotient left in ``action``
    is what motion_penalty sees (a KeyError unless 0 <= q < 4).  A list /
    array of per-slot codes is a deliberate superset (the reference moves the
    robots, then raises in motion_penalty): quotient 0."""
    if action is None:
        return None
    if isinstance(action, (list, tuple, np.ndarray)) and np.ndim(action) > 0:
        a = np.asarray(action, dtype=np.int64).reshape(-1)
        if a.size != n:
            raise ValueError(f"per-slot actions need {n} entries")
        return np.where((a >= 0) & (a < 4), a, 4).astype(np.uint8), 0
    if hasattr(action, "item") and not isinstance(action, (int, np.integer)):
        action = action.item()
    if action == -1:
        return None
    a = int(action)
    digits = np.zeros(n, dtype=np.uint8)
    for i in range(n):
        digits[i] = a % 4
        a //= 4
    if not 0 <= a < 4:
        raise KeyError(a)  # motion_penalty's self.a_inv[a] (:238)
    return digits, a


class SuperGridRL:
    """Drop-in for the reference ``SuperGridRL`` (``super_grid_rl.py:18``)
    whose step/reset run on the GPU.  Same constructor, methods, attributes
    and return types: ``reset -> ((state float64 [P+3, W, L], currstep),
    grid)``, ``step -> ((state, currstep), np.float64 reward, bool done)``
    (the sentinel step returns the int 0 like the reference).  No pygame:
    ``render()`` returns the RGB frame before the reference's cv2 resize."""

    def __init__(self, train_set, env_config, test_set=None, device="cuda", seed=0):
        self._train_gridlis = train_set
        self._test_gridlis = test_set
        self._config = dict(env_config)
        self._numrobot = env_config["numrobot"]
        self._train_maxsteps = env_config["train_maxsteps"]
        self._test_maxsteps = env_config["test_maxsteps"]
        self._collision_penalty = env_config["collision_penalty"]
        self._senseradius = env_config["senseradius"]
        self._free_penalty = env_config["free_penalty"]
        self._done_thresh = env_config["done_thresh"]
        self._done_incr = env_config["done_incr"]
        self._terminal_reward = env_config["terminal_reward"]
        self._dist_r = env_config["dist_reward"]
        self._use_scanning = env_config["use_scanning"]
        self._prev_states = []
        self._device = device
        self._seed = seed
        self._env = None
        self.a_prev = None
        self.reset(False, False)
        self.a_inv = {2: 3, 3: 2, 0: 1, 1: 0}
        self._obs_dim = self._state.shape
        self._num_actions = 4 ** self._numrobot

    # -- device plumbing ---------------------------------------------------
    def _bind_grid(self, grid):
        g = np.asarray(grid, dtype=np.float64)
        if self._env is None or (self._env.width, self._env.length) != g.shape:
            if self._env is not None:
                self._env.close()
            self._env = BatchSuperGridEnv(self._config, 1, [g], device=self._device, seed=self._seed,
                                          auto_reset=False)
        else:
            self._env.set_grids([g])
        torch = self._env._torch
        self._env.set_state(_lib.SG_FIELD_DONE_THRESH, torch.tensor([float(self._done_thresh)], dtype=torch.float64))
        self._env.set_state(_lib.SG_FIELD_A_PREV, torch.tensor([self._a_prev_code()]))

    def _a_prev_code(self):
        return -1 if self.a_prev is None else int(self.a_prev)

    def _pull(self):
        env = self._env
        planes = env.planes[0].cpu().numpy()
        dist = env.dist[0].cpu().numpy()
        pos = env.get_state(_lib.SG_FIELD_POS)[0].cpu().numpy()
        self._xinds = pos[:, 0].astype(int)
        self._yinds = pos[:, 1].astype(int)
        self._currstep = int(env.get_state(_lib.SG_FIELD_CURRSTEP)[0].item())
        self._done_thresh_dev = float(env.get_state(_lib.SG_FIELD_DONE_THRESH)[0].item())
        self._cov_count = int(env.get_state(_lib.SG_FIELD_COV_COUNT)[0].item())
        state = np.empty((planes.shape[0] + 1,) + planes.shape[1:], dtype=np.float64)
        state[:-1] = planes
        state[-1] = dist
        self._state = state
        P = planes.shape[0] - 2
        self._observed_obstacles = state[P]
        self._free = state[P + 1]

    # -- reference API -------------------------------------------------------
    def reset(self, testing, ind):  # :343-399
        if testing and self._test_gridlis is not None:
            grid = self._test_gridlis[ind]
        else:
            grid = self._train_gridlis[np.random.randint(len(self._train_gridlis))]
        self._grid = grid
        self._gridwidth, self._gridlen = grid.shape[0], grid.shape[1]
        W, L = self._gridwidth, self._gridlen
        xs = np.zeros(self._numrobot, dtype=int)
        ys = np.zeros(self._numrobot, dtype=int)
        seen = {}
        count = 0
        while count != self._numrobot:  # the reference's RNG call sequence
            x = np.random.randint(W)
            y = np.random.randint(L)
            if grid[x][y] >= 0 and (x, y) not in seen:
                seen[(x, y)] = 1
                xs[count], ys[count] = x, y
                count += 1
        self._bind_grid(grid)
        pos = np.stack([xs, ys], 1)[None].astype(np.int32)
        self._env.reset(positions=pos)
        self._env.check()
        self._pull()
        return self.get_state(), self._grid

    def step(self, action):  # :74-225
        dec = decode_super_action(action, self._numrobot)
        env = self._env
        torch = env._torch
        if dec is None:
            acts = np.full((1, self._numrobot), 4, dtype=np.uint8)
            acts[0, 0] = _lib.ACT_SENTINEL
            env.step(torch.from_numpy(acts).to(env.device))
            env.check()
            self._pull()
            return self.get_state(), 0, True
        digits, q = dec
        env.step(torch.from_numpy(digits[None]).to(env.device), quot=torch.tensor([q], dtype=torch.int32))
        env.check()
        reward = np.float64(env.reward[0].item())
        done = bool(env.done[0].item())
        self.a_prev = q
        self._pull()
        self._done_thresh = self._done_thresh_dev if done else self._done_thresh
        return self.get_state(), reward, done

    def get_state(self):  # :305-317
        return self._state.copy(), self._currstep

    def get_pos_image(self):  # :319-341
        P = self._state.shape[0] - 3
        return [self._state[p].copy() for p in range(P)]

    def get_distance_map(self):  # :281-303 (of the current state)
        return self._state[-1].astype(np.float32)

    def motion_penalty(self, a):  # :227-243 (pure; step applies it on the device)
        inv = self.a_inv[a]
        if a == self.a_prev:
            return 0
        if a == inv:
            return -2
        return -1

    def isInBounds(self, x, y):  # :245-256
        return x >= 0 and x < self._gridwidth and y >= 0 and y < self._gridlen

    def isOccupied(self, x, y):  # :258-279
        if self._grid[x][y] < 0:
            return True
        return any(a == x and b == y for a, b in zip(self._xinds, self._yinds))

    def done(self):  # :401-414
        if min(self._done_thresh, 1) <= self.percent_covered():
            print("Full Environment Covered")
            self._done_thresh += self._done_incr
            torch = self._env._torch
            self._env.set_state(_lib.SG_FIELD_DONE_THRESH, torch.tensor([float(self._done_thresh)], dtype=torch.float64))
            return True
        return False

    def percent_covered(self):  # :416-421
        return self._cov_count / np.count_nonzero(self._grid > 0)

    def render(self):  # :423-463 up to the cv2 resize / pygame blit
        obst = self._observed_obstacles
        inv_free = 1 - self._free
        pos = self.get_pos_image()[0]
        return (np.stack([200 * obst, 0 * obst, 255 * obst], -1)
                + np.stack([0 * inv_free, 225 * inv_free, 255 * inv_free], -1)
                + np.stack([255 * pos, 0 * pos, 0 * pos], -1))
