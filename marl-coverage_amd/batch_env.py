"""BatchCoverageEnv: many DecGridRL environments stepped by one HIP launch.

PyTorch is used only as the device-memory container: every buffer handed to
libmarlcov.so is a torch CUDA(HIP) tensor passed as a raw pointer, and every
call is enqueued on torch's current stream for the env's device.

Semantics per env are the reference's ``DecGridRL`` (dec_grid_rl.py:21-552);
batch extras are the action bytes of include/marlcov.h (255 in agent 0's byte
= the reference's ``action == None or -1`` path), auto-reset and a device
Philox stream for start cells / synthetic grids.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .sensors import LidarSensor, SquareSensor, make_sensor

_FIELD_DTYPES = {
    _lib.FIELD_POS: "int32", _lib.FIELD_MOVED: "int64", _lib.FIELD_FREE: "int64",
    _lib.FIELD_OBST: "int64", _lib.FIELD_VISITED: "int64", _lib.FIELD_FREE_COUNT: "int32",
    _lib.FIELD_VISITED_COUNT: "int32", _lib.FIELD_CURRSTEP: "int32",
    _lib.FIELD_DONE_THRESH: "float64", _lib.FIELD_ENV_GRID: "int32", _lib.FIELD_EPISODE: "int32",
    _lib.FIELD_NUMFREE: "int32", _lib.FIELD_GRID_NEG: "int64", _lib.FIELD_GRID_POS: "int64",
    _lib.FIELD_DIST_MW: "int32", _lib.FIELD_DIST_LISTED: "int32",
    _lib.FIELD_EP_PC: "float64", _lib.FIELD_EP_LEN: "int32", _lib.FIELD_DJ_LISTED: "int32",
    _lib.FIELD_DIST_CACHED: "int32", _lib.FIELD_DIST_TOTALS: "int64",
}


def pad_grid(grid) -> np.ndarray:
    """The reference's border: np.pad(grid, 1, constant -1) (dec_grid_rl.py:471)."""
    return np.pad(np.asarray(grid, dtype=np.float64), (1,), "constant", constant_values=(-1,))


def grid_to_int8(padded) -> np.ndarray:
    """Padded float grid -> int8 {-1, 0, 1}.

    Every grid source of the reference yields exactly these values (gridgen
    +-1, Utils/gridmaker.py:127; PNG maps clip(img - 1, -1, 1) of uint8,
    :89-91), and the env only ever tests ``< 0`` / ``>= 0`` / ``> 0`` or clips
    to [0, 1] (dec_grid_rl.py:310,498,517,552; lidar.py:52;
    squaresensor.py:34-35), so the bit planes are exact.  Other values are
    rejected rather than silently rounded."""
    g = np.asarray(padded, dtype=np.float64)
    if not np.all((g == -1) | (g == 0) | (g == 1)):
        raise ValueError("grid values must be in {-1, 0, 1} (reference grid semantics)")
    return g.astype(np.int8)


class BatchCoverageEnv:
    """``num_envs`` independent coverage envs on one HIP device.

    Parameters mirror ``DecGridRL(train_set, env_config)``: ``env_config`` is
    the reference dict; ``grids`` a sequence of UNPADDED 2-D grids (the pool;
    env ``e`` starts on grid ``e % len(grids)`` unless ``env_grid`` is given),
    or ``gen=dict(width=, length=, prob_obst=, seed=, num_grids=)`` to draw a
    Bernoulli pool on the device.

    ``step`` / ``reset`` return the env's persistent output tensors (obs uint8
    [B, N, Lc, E, E], reward float64 [B], done uint8 [B]); they are
    overwritten by the next call — clone them to keep them.

    ``env_offset`` / ``grid_offset`` (default: ``env_offset``) are the global
    ids of env 0 and pool grid 0 when this handle is one shard of a larger
    batch: every device random stream is keyed by global id, so
    the shard's envs match the same envs of the whole batch bit for bit.
    """

    def __init__(self, env_config, num_envs, grids=None, *, gen=None, device="cuda",
                 seed=0, auto_reset=True, reset_grid_mode="keep", env_grid=None,
                 sensor=None, want_adjacency=None, env_offset=0, grid_offset=None):
        import torch

        self._torch = torch
        self.lib = _lib.load()
        self.config = dict(env_config)
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("BatchCoverageEnv needs a HIP device (torch 'cuda' device)")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.num_envs = int(num_envs)
        self.num_agents = int(self.config["numrobot"])
        self.sensor = sensor if sensor is not None else make_sensor(self.config)
        ego = int(self.config["egoradius"])
        mini = int(self.config.get("mini_map_rad", 0))
        self.pad = max(ego, mini)

        if (grids is None) == (gen is None):
            raise ValueError("give exactly one of grids= or gen=")
        if grids is not None:
            padded = [pad_grid(g) for g in grids]
            shapes = {p.shape for p in padded}
            if len(shapes) != 1:
                raise ValueError(f"all pool grids must share one shape, got {sorted(shapes)}")
            self.width, self.length = padded[0].shape
            self.num_grids = len(padded)
        else:
            self.width, self.length = int(gen["width"]) + 2, int(gen["length"]) + 2
            self.num_grids = int(gen.get("num_grids", self.num_envs))

        c = _lib.McConfig()
        c.num_envs = self.num_envs
        c.num_agents = self.num_agents
        c.width, c.length = self.width, self.length
        c.num_grids = self.num_grids
        if self.sensor.sensor_type == LidarSensor.sensor_type:
            c.sensor_type = _lib.SENSOR_LIDAR
            c.num_beams = self.sensor._num_lasers
            c.lidar_range = float(self.sensor._max_range)
        elif self.sensor.sensor_type == SquareSensor.sensor_type:
            c.sensor_type = _lib.SENSOR_SQUARE
            c.square_radius = self.sensor._radius
        else:
            raise ValueError(f"unsupported sensor {self.sensor!r}")
        c.egoradius = ego
        c.pad = self.pad
        c.mini_map_rad = mini
        c.collision_penalty = float(self.config["collision_penalty"])
        c.terminal_reward = float(self.config["terminal_reward"])
        c.done_thresh = float(self.config["done_thresh"])
        c.done_incr = float(self.config["done_incr"])
        c.maxsteps = int(self.config["maxsteps"])
        c.comm_radius = int(self.config["comm_radius"])
        c.map_sharing = int(bool(self.config["map_sharing"]))
        c.single_square_tool = int(bool(self.config["single_square_tool"]))
        c.dist_reward = int(bool(self.config.get("dist_reward", 0)))
        c.dijkstra_input = int(bool(self.config.get("dijkstra_input", 0)))
        c.auto_reset = int(bool(auto_reset))
        c.reset_grid_mode = {"keep": 0, "random": 1}[reset_grid_mode]
        c.seed = int(seed) & (2 ** 64 - 1)
        c.env_offset = int(env_offset)
        c.grid_offset = int(env_offset if grid_offset is None else grid_offset)
        self.env_offset = c.env_offset
        self._cfg = c

        handle = ctypes.c_void_p()
        _lib.check(self.lib.mc_create(ctypes.byref(c), dev.index, ctypes.byref(handle)), "mc_create")
        self._h = handle
        lay = _lib.McLayout()
        _lib.check(self.lib.mc_query(self._h, ctypes.byref(lay)), "mc_query")
        self.layout = lay
        self.tile_rows, self.tile_cols = lay.tile_rows, lay.tile_cols
        self.obs_shape = (self.num_agents, lay.obs_layers, lay.obs_side, lay.obs_side)
        self.num_actions = 4

        if self.sensor.sensor_type == LidarSensor.sensor_type:
            self._upload_beams(self.sensor)
            self.sensor.add_listener(self._upload_beams)

        if grids is not None:
            host = np.stack([grid_to_int8(p) for p in padded])
            dgrids = torch.from_numpy(host).to(dev)
            _lib.check(self.lib.mc_set_grids(self._h, dgrids.data_ptr(), self.num_grids, self._stream()),
                       "mc_set_grids")
        else:
            _lib.check(self.lib.mc_generate_grids(self._h, int(gen.get("seed", 0)),
                                                  float(gen["prob_obst"]), self._stream()),
                       "mc_generate_grids")
        if env_grid is not None:
            self.set_env_grids(env_grid)

        B, N = self.num_envs, self.num_agents
        self.obs = torch.zeros((B,) + self.obs_shape, dtype=torch.uint8, device=dev)
        self.reward = torch.zeros(B, dtype=torch.float64, device=dev)
        self.done = torch.zeros(B, dtype=torch.uint8, device=dev)
        if want_adjacency is None:
            want_adjacency = bool(self.config.get("allow_comm", 0))
        self.adj = torch.zeros((B, N, N), dtype=torch.uint8, device=dev) if want_adjacency else None
        # dist_reward: the float32 distance-map crop (obs layer 3), written by
        # every reset / step next to the uint8 obs (include/marlcov.h)
        self.dist_obs = None
        if c.dist_reward:
            E = lay.obs_side
            self.dist_obs = torch.zeros((B, N, E, E), dtype=torch.float32, device=dev)
            _lib.check(self.lib.mc_set_dist_obs(self._h, self.dist_obs.data_ptr()), "mc_set_dist_obs")
        # mini_map_rad: the float64 minimap layers (obs layers 3 and 4)
        self.minimap_obs = None
        if mini > 0:
            E = lay.obs_side
            self.minimap_obs = torch.zeros((B, N, 2, E, E), dtype=torch.float64, device=dev)
            _lib.check(self.lib.mc_set_minimap_obs(self._h, self.minimap_obs.data_ptr()), "mc_set_minimap_obs")

    # ------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(self._torch.cuda.current_stream(self.device).cuda_stream)

    def _upload_beams(self, sensor):
        if not getattr(self, "_h", None):  # closed
            return
        tab = np.ascontiguousarray(sensor.table(), dtype=np.float64)
        _lib.check(self.lib.mc_set_beam_table(self._h, tab.ctypes.data, tab.shape[0]),
                   "mc_set_beam_table")
        self._cfg.num_beams = tab.shape[0]  # only once the device holds the table

    def _adj_ptr(self):
        return None if self.adj is None else self.adj.data_ptr()

    def close(self):
        if getattr(self, "_h", None):
            if getattr(getattr(self, "sensor", None), "sensor_type", None) == LidarSensor.sensor_type:
                self.sensor.remove_listener(self._upload_beams)
            self.lib.mc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------
    def set_env_grids(self, env_grid):
        t = self._torch.as_tensor(np.asarray(env_grid, dtype=np.int32), device=self.device)
        if t.numel() != self.num_envs or int(t.min()) < 0 or int(t.max()) >= self.num_grids:
            raise ValueError("env_grid must hold num_envs indices into the grid pool")
        _lib.check(self.lib.mc_set_env_grids(self._h, t.data_ptr(), self._stream()), "mc_set_env_grids")

    def reset(self, env_mask=None, positions=None):
        """Reset the envs in ``env_mask`` (bool/uint8 [B], None = all).
        ``positions`` int32 [B, N, 2] (padded coords) injects start cells,
        else they are drawn on the device.  Returns obs (and adjacency)."""
        torch = self._torch
        m = None
        if env_mask is not None:
            m = torch.as_tensor(env_mask, device=self.device).to(torch.uint8).contiguous()
        p = None
        if positions is not None:
            p = torch.as_tensor(positions, device=self.device).to(torch.int32).contiguous()
            if tuple(p.shape) != (self.num_envs, self.num_agents, 2):
                raise ValueError("positions must be [num_envs, numrobot, 2]")
        _lib.check(self.lib.mc_reset(self._h, None if m is None else m.data_ptr(),
                                     None if p is None else p.data_ptr(), self.obs.data_ptr(),
                                     self._adj_ptr(), self._stream()), "mc_reset")
        if self.adj is not None:
            return self.obs, self.adj
        return self.obs

    def step(self, actions):
        """``actions``: uint8 [B, N] device tensor of per-agent codes (0 +x,
        1 +y, 2 -x, 3 -y, 4..254 no-op, 255 in agent 0 = sentinel step)."""
        torch = self._torch
        a = actions
        if not (isinstance(a, torch.Tensor) and a.dtype == torch.uint8 and a.device == self.device
                and a.is_contiguous()):
            a = torch.as_tensor(a, device=self.device).to(torch.uint8).contiguous()
        if tuple(a.shape) != (self.num_envs, self.num_agents):
            raise ValueError(f"actions must be [{self.num_envs}, {self.num_agents}] uint8")
        _lib.check(self.lib.mc_step(self._h, a.data_ptr(), self.reward.data_ptr(), self.done.data_ptr(),
                                    self.obs.data_ptr(), self._adj_ptr(), self._stream()), "mc_step")
        if self.adj is not None:
            return (self.obs, self.adj), self.reward, self.done
        return self.obs, self.reward, self.done

    def rollout(self, actions):
        """Step K times with known actions, one C-ABI call (mc_step_many):
        ``actions`` uint8 [K, B, N] device tensor; returns new tensors obs
        [K, B, N, Lc, E, E], reward [K, B], done [K, B] -- step k's outputs,
        exactly what K ``step`` calls would have returned, with the per-step
        adjacency [K, B, N, N] as ``((obs, adj), reward, done)`` when the env
        returns it.  Configs with float obs layers (dist_reward, minimap) keep
        one registered float buffer per env (mc_set_dist_obs /
        mc_set_minimap_obs), so their per-step float layers cannot come back
        from one call: use ``step`` for them."""
        torch = self._torch
        if self.dist_obs is not None or self.minimap_obs is not None:
            raise ValueError("rollout: dist_reward / mini_map_rad configs write their float obs layers to one "
                             "registered buffer; step() returns them per step")
        a = actions
        if not (isinstance(a, torch.Tensor) and a.dtype == torch.uint8 and a.device == self.device
                and a.is_contiguous()):
            a = torch.as_tensor(a, device=self.device).to(torch.uint8).contiguous()
        if a.dim() != 3 or tuple(a.shape[1:]) != (self.num_envs, self.num_agents):
            raise ValueError(f"actions must be [K, {self.num_envs}, {self.num_agents}] uint8")
        K = a.shape[0]
        obs = torch.empty((K,) + tuple(self.obs.shape), dtype=torch.uint8, device=self.device)
        rew = torch.empty((K, self.num_envs), dtype=torch.float64, device=self.device)
        done = torch.empty((K, self.num_envs), dtype=torch.uint8, device=self.device)
        adj = None
        if self.adj is not None:
            adj = torch.empty((K,) + tuple(self.adj.shape), dtype=self.adj.dtype, device=self.device)
        if K > 0:
            _lib.check(self.lib.mc_step_many(self._h, a.data_ptr(), a[0].numel(), K, rew.data_ptr(),
                                             rew[0].numel() * 8, done.data_ptr(), done[0].numel(), obs.data_ptr(),
                                             obs[0].numel(), adj.data_ptr() if adj is not None else None,
                                             adj[0].numel() if adj is not None else 0, self._stream()),
                       "mc_step_many")
            self.obs.copy_(obs[-1])
            self.reward.copy_(rew[-1])
            self.done.copy_(done[-1])
            if adj is not None:
                self.adj.copy_(adj[-1])
        if adj is not None:
            return (obs, adj), rew, done
        return obs, rew, done

    def step_many_raw(self, actions_ptr: int, actions_stride: int, num_steps: int, reward_ptr: int,
                      done_ptr: int, obs_ptr: int, stream: int):
        """Benchmarks: ``num_steps`` launches in one C call (mc_step_many),
        actions at ``actions_ptr + k * actions_stride``, every step's outputs
        into the same buffers."""
        return self.lib.mc_step_many(self._h, actions_ptr, actions_stride, num_steps, reward_ptr, 0, done_ptr, 0,
                                     obs_ptr, 0, None, 0, stream)

    def random_actions(self, seed, step, out=None):
        """uint8 [B, N] actions uniform in {0..3} from Philox(seed, global env
        id, step) (mc_random_actions): the same bytes for an env whatever the
        shard it is stepped in."""
        torch = self._torch
        if out is None:
            out = torch.empty((self.num_envs, self.num_agents), dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.mc_random_actions(self._h, int(seed) & (2 ** 64 - 1), int(step), out.data_ptr(),
                                              self._stream()), "mc_random_actions")
        return out

    def kernel_variant(self) -> str:
        """The env-kernel instantiation mc_step launches (mc_kernel_variant)."""
        return self.lib.mc_kernel_variant(self._h).decode()

    def step_raw(self, actions_ptr: int, reward_ptr: int, done_ptr: int, obs_ptr: int, stream: int):
        """Zero-overhead launch for benchmarks: raw device pointers / stream."""
        return self.lib.mc_step(self._h, actions_ptr, reward_ptr, done_ptr, obs_ptr, None, stream)

    # ------------------------------------------------------------------
    def field_shape(self, field):
        B, N, G = self.num_envs, self.num_agents, self.num_grids
        mw = (self.tile_rows // 4, self.tile_cols // 4, 4, 4)  # 4x4 blocks of 8x8-cell tiles (tiles.py)
        return {
            _lib.FIELD_POS: (B, N, 2), _lib.FIELD_MOVED: (B,), _lib.FIELD_FREE: (B, N) + mw,
            _lib.FIELD_OBST: (B, N) + mw, _lib.FIELD_VISITED: (B,) + mw, _lib.FIELD_FREE_COUNT: (B,),
            _lib.FIELD_VISITED_COUNT: (B,), _lib.FIELD_CURRSTEP: (B,), _lib.FIELD_DONE_THRESH: (B,),
            _lib.FIELD_ENV_GRID: (B,), _lib.FIELD_EPISODE: (B,), _lib.FIELD_NUMFREE: (G,),
            _lib.FIELD_GRID_NEG: (G,) + mw, _lib.FIELD_GRID_POS: (G,) + mw,
            _lib.FIELD_DIST_MW: (B, N, 2), _lib.FIELD_DIST_LISTED: (1,),
            _lib.FIELD_EP_PC: (B,), _lib.FIELD_EP_LEN: (B,), _lib.FIELD_DJ_LISTED: (1,),
            _lib.FIELD_DIST_CACHED: (1,), _lib.FIELD_DIST_TOTALS: (4,),
        }[field]

    def get_state(self, field, out=None):
        """Device copy of one state field (`out`: a device tensor of the field's
        shape and dtype to fill instead of a new one)."""
        torch = self._torch
        if out is None:
            t = torch.empty(self.field_shape(field), dtype=getattr(torch, _FIELD_DTYPES[field]),
                            device=self.device)
        else:
            t = out
            if (tuple(t.shape) != self.field_shape(field) or t.dtype != getattr(torch, _FIELD_DTYPES[field])
                    or t.device != torch.device(self.device) or not t.is_contiguous()):
                raise ValueError(f"out for field {field} must be a contiguous {_FIELD_DTYPES[field]} "
                                 f"tensor of shape {self.field_shape(field)} on {self.device}")
        nbytes = t.numel() * t.element_size()
        _lib.check(self.lib.mc_get_state(self._h, field, t.data_ptr(), nbytes, self._stream()),
                   "mc_get_state")
        return t

    def set_state(self, field, tensor):
        torch = self._torch
        t = tensor.to(self.device).to(getattr(torch, _FIELD_DTYPES[field])).contiguous()
        if tuple(t.shape) != self.field_shape(field):
            raise ValueError(f"field {field} must have shape {self.field_shape(field)}")
        nbytes = t.numel() * t.element_size()
        _lib.check(self.lib.mc_set_state(self._h, field, t.data_ptr(), nbytes, self._stream()),
                   "mc_set_state")

    def percent_covered(self):
        """float64 [B]: count_nonzero(_free_pad > 0) / count_nonzero(grid > 0)
        (dec_grid_rl.py:548-552; summed over agents, can exceed 1)."""
        fc = self.get_state(_lib.FIELD_FREE_COUNT).to(self._torch.float64)
        nf = self.get_state(_lib.FIELD_NUMFREE).to(self._torch.float64)
        eg = self.get_state(_lib.FIELD_ENV_GRID).long()
        return fc / nf[eg]

    def check(self):
        """Synchronise and raise if a kernel flagged a device error."""
        _lib.check(self.lib.mc_check(self._h, self._stream()), "mc_check")
