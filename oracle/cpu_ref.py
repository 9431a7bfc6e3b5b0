"""CPU oracle for the DecGridRL step/reset hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
*checker* (or as the timed CPU baseline).  The product path in
``marl-coverage_amd/`` never imports it and fails loudly when its HIP library
is missing.

What it is: a NumPy restatement of the reference environment
``Environments/dec_grid_rl.py:DecGridRL`` (ExistentialRobotics/MARL-Coverage)
and its sensors ``Environments/Sensors/lidar.py`` / ``squaresensor.py``,
keeping the reference's float64 state arrays, its per-robot full-map copies
and its per-cell Python beam march, so it is also a fair stand-in for the
reference's own CPU step when timed (bench.py ``cpu_baseline.kind = "port"``).
Every function cites the reference lines it restates.

Pinning: ``tests/test_oracle_golden.py`` checks this module bit-for-bit
against golden vectors captured from the real reference in the build
container (``tests/golden/make_golden.py``: reference imported with
``pygame``/``cv2`` stubs).  Two pieces are pinned only against the reference's
own code paths with a restated third-party call, not against the third-party
library itself:
  * ``dist_reward`` uses ``cv2.distanceTransform(DIST_L1, DIST_MASK_PRECISE)``
    (``dec_grid_rl.py:273-275``); cv2 is not installed, so both the oracle and
    the golden capture use the exact-L1 SciPy restatement below.  Parity with
    real OpenCV: *unpinned*.
  * ``mini_map_rad > 0`` uses ``cv2.resize(INTER_LINEAR)``
    (``dec_grid_rl.py:360-370``); ``cv2_resize_linear`` restates OpenCV's
    generic CV_64F path (the golden capture uses the same restatement).
    Parity with real OpenCV: *unpinned*.
"""
from __future__ import annotations

import heapq

import numpy as np


# --------------------------------------------------------------------------
# sensors
# --------------------------------------------------------------------------
def lidar_thetas(num_lasers: int) -> np.ndarray:
    """Beam angles, ``lidar.py:14`` (even counts allowed)."""
    return np.linspace(0, 2 * np.pi, num=num_lasers, endpoint=False)


def lidar_beam_table(thetalist) -> np.ndarray:
    """[B, 3] float64 (xinc, yinc, distinc) per beam, ``lidar.py:38-48``.

    Evaluated per scalar theta with NumPy scalar ops, exactly the expression
    sequence the reference runs inside ``getMeasurement``.
    """
    out = np.empty((len(thetalist), 3), dtype=np.float64)
    for k, theta in enumerate(thetalist):
        xi = np.cos(theta)
        yi = np.sin(theta)
        larger = max(abs(xi), abs(yi))
        xi /= larger
        yi /= larger
        out[k, 0] = xi
        out[k, 1] = yi
        out[k, 2] = np.sqrt(xi ** 2 + yi ** 2)
    return out


class LidarRef:
    """Restates ``LidarSensor`` (``lidar.py:5-68``)."""

    kind = "lidar"

    def __init__(self, sensor_config, allow_even=False):
        self._num_lasers = sensor_config["num_lasers"]
        self._max_range = sensor_config["range"]
        if not allow_even:
            assert self._num_lasers % 2 == 1, "odd number of lasers needed"  # lidar.py:11
        self._thetalist = lidar_thetas(self._num_lasers)
        self._table = lidar_beam_table(self._thetalist)

    def set_thetalist(self, thetalist):
        self._thetalist = np.asarray(thetalist, dtype=np.float64)
        self._num_lasers = len(self._thetalist)
        self._table = lidar_beam_table(self._thetalist)

    def getMeasurement(self, x, y, oc, free_map, obst_map, pad):
        """``lidar.py:16-65``: copy both maps, march every beam.  The beam
        increments are derived per call from the angle, as the reference does
        (``:38-48``; the same expressions as ``lidar_beam_table``, so the same
        bits), and the bound test is a method call (``:67-68``): the port's
        per-step cost stays the reference's (the bench's CPU baseline,
        ``tools/calibrate_cpu.py``)."""
        width, length = np.shape(oc)
        new_free = np.copy(free_map)
        new_obst = np.copy(obst_map)
        rng = self._max_range
        inside = self.inbounds
        for theta in self._thetalist:
            px = x
            py = y
            xinc = np.cos(theta)
            yinc = np.sin(theta)
            larger = max(abs(xinc), abs(yinc))
            xinc /= larger
            yinc /= larger
            dinc = np.sqrt(xinc ** 2 + yinc ** 2)
            travelled = 0
            while inside(px, py, length, width) and oc[int(px), int(py)] >= 0 and travelled < rng:
                new_free[int(px) + pad, int(py) + pad] = 1
                px += xinc
                py += yinc
                travelled += dinc
            if inside(px, py, length, width) and oc[int(px), int(py)] >= 0:
                new_free[int(px) + pad, int(py) + pad] = 1
            else:
                new_obst[int(px) + pad, int(py) + pad] = 1
        return new_free, new_obst

    @staticmethod
    def inbounds(px, py, length, width):
        """``lidar.py:67-68``."""
        return px >= 0 and py >= 0 and px < width and py < length


class SquareRef:
    """Restates ``SquareSensor`` (``squaresensor.py:4-37``)."""

    kind = "square_sensor"

    def __init__(self, sensor_config):
        self._radius = sensor_config["range"]

    def getMeasurement(self, x, y, oc, free_map, obst_map, pad):
        new_free = free_map.copy()
        new_obst = obst_map.copy()
        r = self._radius
        x0, x1 = max(x - r, 0), min(x + r + 1, oc.shape[0])
        y0, y1 = max(y - r, 0), min(y + r + 1, oc.shape[1])
        seen = oc[x0:x1, y0:y1]
        new_free[x0 + pad:x1 + pad, y0 + pad:y1 + pad] = np.clip(seen, 0, 1)
        new_obst[x0 + pad:x1 + pad, y0 + pad:y1 + pad] = np.clip(-seen, 0, 1)
        return new_free, new_obst


# --------------------------------------------------------------------------
# auxiliary observation layers
# --------------------------------------------------------------------------
def l1_distance_to_covered(free: np.ndarray) -> np.ndarray:
    """Restated ``cv2.distanceTransform(inv, DIST_L1, DIST_MASK_PRECISE)``.

    ``inv`` is 1 on uncovered cells (``dec_grid_rl.py:273``).  Exact L1 distance
    of every uncovered cell to the nearest covered cell, float32; with no
    covered cell at all we return the SciPy convention (-1) — unpinned.
    """
    from scipy.ndimage import distance_transform_cdt

    inv = (free == 0).astype(np.uint8)
    return distance_transform_cdt(inv, metric="taxicab").astype(np.float32)


def _linear_taps(src_n: int, dst_n: int):
    """OpenCV's INTER_LINEAR tap tables (resizeGeneric_ set-up in
    imgproc/src/resize.cpp, non-area mode): per destination index the source
    index, the float32 weights (1 - f, f), and ``xmax`` (from there on the
    horizontal pass copies ``S[xofs]``).  ``inv_scale = dst/src`` and
    ``scale = 1/inv_scale`` in double, ``f = (float)((d + 0.5)*scale - 0.5)``,
    ``s = floor(f)``, ``f -= s`` in float; the horizontal indices are clamped
    (s < 0 -> 0, f = 0; s >= n - 1 -> n - 1, f = 0), the vertical ones are
    clipped when rows are fetched."""
    inv_scale = dst_n / src_n
    scale = 1.0 / inv_scale
    xofs, yofs, alpha, beta = [], [], [], []
    xmax = dst_n
    for d in range(dst_n):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        yofs.append(s)
        beta.append((np.float32(np.float32(1.0) - f), f))
        fx, sx = f, s
        if sx < 0:
            fx, sx = np.float32(0.0), 0
        if sx + 1 >= src_n:
            xmax = min(xmax, d)
            if sx >= src_n - 1:
                fx, sx = np.float32(0.0), src_n - 1
        xofs.append(sx)
        alpha.append((np.float32(np.float32(1.0) - fx), fx))
    return xofs, alpha, xmax, yofs, beta


def cv2_resize_linear(src: np.ndarray, dst_n: int) -> np.ndarray:
    """Restated ``cv2.resize(src, (dst_n, dst_n), interpolation=INTER_LINEAR)``
    for a square float64 image (``dec_grid_rl.py:365-370``): OpenCV's generic
    path for CV_64F, ``HResizeLinear<double, double, float>`` then
    ``VResizeLinear<double, double, float>`` — double arithmetic with float
    weights, horizontal pass first, no FMA.  cv2 is absent: parity with real
    OpenCV (its version, IPP/HAL dispatch) is *unpinned*."""
    n = src.shape[0]
    if src.shape != (n, n):
        raise ValueError("square source expected")
    if dst_n == n:  # cv::resize copies when the sizes match
        return src.astype(np.float64).copy()
    xofs, alpha, xmax, yofs, beta = _linear_taps(n, dst_n)
    h = np.empty((n, dst_n))
    for r in range(n):
        row = src[r]
        for d in range(dst_n):
            sx = xofs[d]
            if d < xmax:
                h[r, d] = float(row[sx]) * float(alpha[d][0]) + float(row[sx + 1]) * float(alpha[d][1])
            else:
                h[r, d] = float(row[sx])
    out = np.empty((dst_n, dst_n))
    for d in range(dst_n):
        r0 = min(max(yofs[d], 0), n - 1)
        r1 = min(max(yofs[d] + 1, 0), n - 1)
        b0, b1 = float(beta[d][0]), float(beta[d][1])
        for c in range(dst_n):
            out[d, c] = h[r0, c] * b0 + h[r1, c] * b1
    return out


def distance_map(free: np.ndarray) -> np.ndarray:
    """``DecGridRL.get_distance_map`` (``dec_grid_rl.py:260-282``)."""
    d = l1_distance_to_covered(free)
    if np.max(d) > 0:
        d = d / np.max(d)
    return 1 - d


def _open_neighbours(x, y, grid, seen):
    """``dijkstra.py:31-60``: +x, -x, +y, -y; unvisited and not -1."""
    h, w = grid.shape
    out = []
    for nx, ny in ((x + 1, y), (x - 1, y), (x, y + 1), (x, y - 1)):
        if 0 <= nx < h and 0 <= ny < w and seen[nx][ny] == 0 and grid[nx][ny] != -1:
            out.append((nx, ny))
    return out


def dijkstra_path_map(grid, sx, sy):
    """``dijkstra.py:112-187``: path (1s) from start to the nearest 0 cell.

    ``queue.PriorityQueue`` of ``(cost, (x, y))`` tuples == a heap of the same
    tuples, so tie order is (cost, x, y).
    """
    heap = [(0, (sx, sy))]
    seen = np.zeros(grid.shape)
    cost = -1 * np.ones(grid.shape)
    goal = None
    while heap:
        c, (cx, cy) = heapq.heappop(heap)
        if seen[cx][cy] == 1:
            continue
        seen[cx][cy] = 1
        cost[cx][cy] = c
        if grid[cx][cy] == 0:
            goal = (cx, cy)
            break
        for nb in _open_neighbours(cx, cy, grid, seen):
            heapq.heappush(heap, (c + 1, nb))
    path = np.zeros(grid.shape)
    if goal is None:
        return path
    cur = goal
    cur_cost = cost[cur[0], cur[1]]
    path[cur[0], cur[1]] = 1
    back = 1 - seen
    while cur[0] != sx or cur[1] != sy:
        for nb in _open_neighbours(cur[0], cur[1], grid, back):
            if cost[nb[0], nb[1]] == cur_cost - 1:
                cur_cost -= 1
                cur = nb
                break
        path[cur[0], cur[1]] = 1
    assert path[sx, sy] == 1
    return path


# --------------------------------------------------------------------------
# the environment
# --------------------------------------------------------------------------
def make_sensor(env_config):
    kind = env_config["sensor_type"]
    if kind == "lidar":
        return LidarRef(env_config["sensor_config"],
                        allow_even=bool(env_config.get("allow_even_beams", False)))
    if kind == "square_sensor":
        return SquareRef(env_config["sensor_config"])
    raise ValueError(f"unknown sensor_type {kind!r}")


class DecGridRLRef:
    """Restates ``DecGridRL`` (``dec_grid_rl.py:21-552``) minus rendering.

    Same constructor, method names, attribute names and return types.  Extra
    (oracle-only): ``reset(..., positions=[(x, y), ...])`` injects start cells
    instead of drawing them, and ``snapshot()`` exports comparable state.
    """

    def __init__(self, train_set, env_config, use_graph=False, test_set=None):
        self._train_gridlis = train_set
        self._test_gridlis = test_set
        c = env_config
        self._numrobot = c["numrobot"]
        self._maxsteps = c["maxsteps"]
        self._collision_penalty = c["collision_penalty"]
        self._done_thresh = c["done_thresh"]
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
        self._pad = max(self._egoradius, self._mini_map_rad)          # :78
        self.reset(False, None)                                          # :81
        self._obs_dim = self.get_egocentric_observations()[0].shape    # :84
        self._num_actions = 4                                            # :85

    # ---- step ------------------------------------------------------------
    def step(self, action):
        """``dec_grid_rl.py:91-169``."""
        done = False
        if action is None or (not isinstance(action, np.ndarray) and action == -1) or \
                (isinstance(action, np.ndarray) and action.size == 1 and action == -1):
            done = True
            reward = 0
        else:
            if type(action) != np.ndarray:                              # :110-115
                ulis = np.zeros((self._numrobot,))
                for i in range(self._numrobot):
                    ulis[i] = action % 4
                    action = action // 4
            else:
                ulis = action
            reward = 0
            if self._map_sharing:                                        # :124-125
                self.shareMaps()
            deltas = {0: (1, 0), 1: (0, 1), 2: (-1, 0), 3: (0, -1)}      # :131-145
            for i in range(self._numrobot):
                u = ulis[i]
                for code, (dx, dy) in deltas.items():
                    if u == code:
                        reward += self.updateRobotPos(self._xinds[i] + dx,
                                                      self._yinds[i] + dy, i)
                        break
            self.updateCommmunicationGraph()                             # :148
            reward += self.observe()                                     # :151
            self._currstep += 1                                          # :154
            if min(self._done_thresh, 1) <= self.percent_covered():     # :156-157
                reward += self._terminal_reward
        observations = self.get_egocentric_observations()               # :160
        if done is False:
            done = self.done()                                           # :163-164
        if self._allow_comm and self._use_graph:                         # :166-169
            return [observations, self._adjacency_matrix], reward, done
        return observations, reward, done

    def updateRobotPos(self, x, y, i):
        """``dec_grid_rl.py:171-204``: sequential, occupancy updated at once."""
        if self.isInBounds(x, y) and not self.isOccupied(x, y):
            ox, oy = self._xinds[i], self._yinds[i]
            p = self._pad
            self._robot_pos_map[ox][oy] = 0
            self._robot_pad[ox + p][oy + p] = 0
            self._xinds[i] = x
            self._yinds[i] = y
            self._robot_pos_map[x][y] = 1
            self._robot_pad[x + p][y + p] = 1
            return 0
        return -self._collision_penalty

    def observe(self):
        """``dec_grid_rl.py:206-258``."""
        gained = 0
        p = self._pad
        for i in range(self._numrobot):
            x, y = self._xinds[i], self._yinds[i]
            if self._dist_r:
                dmap = distance_map(self._free_pad[i])
            nf, no = self._sensor.getMeasurement(x, y, self._grid, self._free_pad[i],
                                                 self._obst_pad[i], p)
            self._obst_pad[i] = no
            if self._single_square_tool:
                self._free_pad[i][x + p][y + p] = 1
            else:
                self._free_pad[i] = nf
            if self._dist_r:
                gained += dmap[x, y]          # pad-offset quirk kept (:240)
        before = np.sum(self._visited)
        vis = np.clip(np.sum(self._free_pad, axis=0), 0, 1)
        obs = np.clip(np.sum(self._obst_pad, axis=0), 0, 1)
        self._visited = vis[p:p + self._gridwidth, p:p + self._gridlen]
        self._observed_obstacles = obs[p:p + self._gridwidth, p:p + self._gridlen]
        gained += np.sum(self._visited) - before
        return gained

    def get_distance_map(self, free):
        return distance_map(free)

    def isInBounds(self, x, y):
        """``dec_grid_rl.py:284-295``."""
        return x >= 0 and x < self._gridwidth and y >= 0 and y < self._gridlen

    def isOccupied(self, x, y):
        """``dec_grid_rl.py:297-310``."""
        return self._grid[x][y] < 0 or self._robot_pos_map[x][y] == 1

    def get_egocentric_observations(self):
        """``dec_grid_rl.py:312-372``."""
        layers = 5 if self._mini_map_rad > 0 else 3
        layers += 1 if self._dist_r else 0
        layers += 1 if self._dijkstra_input else 0
        e = self._egoradius
        z = np.zeros((self._numrobot, layers, 2 * e + 1, 2 * e + 1))
        p = self._pad
        for i in range(self._numrobot):
            x, y = self._xinds[i], self._yinds[i]
            z[i][0] = self.arraySubset(self._robot_pad, x, y, e)
            z[i][1] = self.arraySubset(self._free_pad[i], x, y, e)
            z[i][2] = self.arraySubset(self._obst_pad[i], x, y, e)
            if self._dist_r:
                z[i][3] = self.arraySubset(distance_map(self._free_pad[i]), x, y, e)
            if self._dijkstra_input:
                path = dijkstra_path_map(self._free_pad[i] - self._obst_pad[i],
                                         x + p, y + p)
                z[i][3] = self.arraySubset(path, x, y, e)
            if self._mini_map_rad > 0:  # :360-370, overwrites layers 3 and 4
                m = self._mini_map_rad
                z[i][3] = cv2_resize_linear(self.arraySubset(self._free_pad[i], x, y, m), 2 * e + 1)
                z[i][4] = cv2_resize_linear(self.arraySubset(self._obst_pad[i], x, y, m), 2 * e + 1)
        return z

    def updateCommmunicationGraph(self):
        """``dec_grid_rl.py:374-391``: Chebyshev distance <= comm_radius."""
        n = self._numrobot
        adj = np.zeros((n, n))
        for i in range(n):
            for j in range(i, n):
                d = max(abs(self._xinds[i] - self._xinds[j]),
                        abs(self._yinds[i] - self._yinds[j]))
                if d <= self._comm_radius:
                    adj[i][j] = 1
                    adj[j][i] = 1
        self._adjacency_matrix = adj

    def arraySubset(self, array, x, y, radius):
        """``dec_grid_rl.py:393-421``."""
        p = self._pad
        return array[x - radius + p:x + radius + 1 + p, y - radius + p:y + radius + 1 + p]

    def shareMaps(self):
        """``dec_grid_rl.py:423-447``: OR over {j : adj[i][j] or i == j}."""
        n = self._numrobot
        shape = self._free_pad.shape
        ob = np.zeros(shape)
        fr = np.zeros(shape)
        for i in range(n):
            for j in range(n):
                if self._adjacency_matrix[i][j] or i == j:
                    ob[i] += self._obst_pad[j]
                    fr[i] += self._free_pad[j]
        self._obst_pad = np.clip(ob, 0, 1)
        self._free_pad = np.clip(fr, 0, 1)

    # ---- reset -----------------------------------------------------------
    def reset(self, testing, ind, positions=None):
        """``dec_grid_rl.py:449-531``.  ``positions`` (oracle-only) skips the
        rejection draw and places robot i at ``positions[i]`` (padded coords)."""
        if testing and self._test_gridlis is not None:
            g = self._test_gridlis[ind]
        else:
            g = self._train_gridlis[np.random.randint(len(self._train_gridlis))]
        self._grid = np.pad(g, (1,), "constant", constant_values=(-1,))
        self._gridwidth, self._gridlen = self._grid.shape
        self._currstep = 0
        n = self._numrobot
        self._xinds = np.zeros(n, dtype=int)
        self._yinds = np.zeros(n, dtype=int)
        p = self._pad
        W, L = self._gridwidth, self._gridlen
        self._robot_pos_map = np.zeros((W, L))
        self._robot_pad = np.zeros((W + 2 * p, L + 2 * p))
        if positions is not None:
            for k, (x, y) in enumerate(positions):
                assert self._grid[x][y] >= 0 and self._robot_pos_map[x][y] == 0
                self._robot_pos_map[x][y] = 1
                self._xinds[k], self._yinds[k] = x, y
        else:
            placed = 0
            while placed != n:                                           # :491-502
                x = np.random.randint(W)
                y = np.random.randint(L)
                if self._grid[x][y] >= 0 and self._robot_pos_map[x][y] == 0:
                    self._robot_pos_map[x][y] = 1
                    self._xinds[placed] = x
                    self._yinds[placed] = y
                    placed += 1
        self._observed_obstacles = np.zeros((W, L))
        self._obst_pad = np.zeros((n, W + 2 * p, L + 2 * p))
        self._free_pad = np.zeros((n, W + 2 * p, L + 2 * p))
        self._visited = np.zeros((W, L))
        self._numfree = np.count_nonzero(self._grid > 0)
        self._numobserved = 0
        self.updateCommmunicationGraph()
        self.observe()
        observations = self.get_egocentric_observations()
        if self._allow_comm and self._use_graph:
            return observations, self._grid, self._adjacency_matrix
        return observations, self._grid

    def done(self):
        """``dec_grid_rl.py:533-546`` (the print is dropped)."""
        if min(self._done_thresh, 1) <= self.percent_covered():
            self._done_thresh += self._done_incr
            return True
        if self._currstep == self._maxsteps:
            return True
        return False

    def percent_covered(self):
        """``dec_grid_rl.py:548-552``: sum over robots / free cells (may exceed 1)."""
        return np.count_nonzero(self._free_pad > 0) / np.count_nonzero(self._grid > 0)

    # ---- oracle-only helpers ---------------------------------------------
    def snapshot(self):
        """Comparable state: positions, 0/1 maps (as uint8), counters."""
        return {
            "xinds": self._xinds.copy(),
            "yinds": self._yinds.copy(),
            "free_pad": (self._free_pad > 0).astype(np.uint8),
            "obst_pad": (self._obst_pad > 0).astype(np.uint8),
            "robot_pad": (self._robot_pad > 0).astype(np.uint8),
            "visited": (self._visited > 0).astype(np.uint8),
            "adjacency": self._adjacency_matrix.copy(),
            "currstep": int(self._currstep),
            "done_thresh": float(self._done_thresh),
        }
