"""CPU oracle for the centralized SuperGridRL step/reset.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
*checker* (or as the timed CPU baseline).  The product path in
``marl-coverage_amd/`` never imports it.

What it is: a NumPy restatement of ``Environments/super_grid_rl.py:SuperGridRL``
(ExistentialRobotics/MARL-Coverage), keeping the reference's float64 state
arrays and per-cell Python sense loop, so it is also a fair stand-in for the
reference's own CPU step when timed.  Every method cites the lines it
restates.

Pinning: ``tests/test_oracle_golden.py`` replays the fixtures that
``tests/golden/make_golden_super.py`` captured from the real reference class
(imported with ``pygame``/``cv2`` stubs) bit for bit.  ``get_state`` always
calls ``cv2.distanceTransform`` (``super_grid_rl.py:294-296``); cv2 is absent,
so the oracle and the capture share the exact-L1 SciPy restatement below and
parity with real OpenCV is *unpinned* (as for DecGridRL's dist_reward).

Reference behaviour kept on purpose (all probed against the reference):
  * ``ulis`` comes from base-4 digits of the joint int, robot slot 0 = least
    significant digit (:93-98); ``motion_penalty`` then sees the *quotient*
    ``action // 4**N`` (the loop reassigns ``action``, :98,203), i.e. 0 for every
    in-range joint action: -1 per reward slot on the first step of the
    object's life (``a_prev`` is None), 0 afterwards; ``a_prev`` survives
    ``reset`` (:57,208).  A quotient >= 4 raises KeyError (:238).
  * moves: 0 = x-1, 1 = x+1, 2 = y+1, 3 = y-1 (:131-174), unpadded bounds.
  * ``use_scanning``: slot i drives the robot with the i-th smallest
    ``x + y*W`` of the pre-move positions (:108-129).
  * reward slots are summed with ``np.sum`` (:214); no ``maxsteps`` in
    ``done()`` (:401-414).
"""
from __future__ import annotations

from queue import PriorityQueue

import numpy as np


def l1_distance_to_uncovered(free: np.ndarray) -> np.ndarray:
    """Restated ``cv2.distanceTransform(~free, DIST_L1, DIST_MASK_PRECISE)``
    of ``super_grid_rl.py:294-296``: exact L1 distance (float32) of every
    covered cell (``free == 0``) to the nearest cell with ``free != 0``
    (uncovered or obstacle: obstacles are never sensed, so their ``_free``
    stays 1).  No such cell at all: SciPy's convention (-1), unpinned."""
    from scipy.ndimage import distance_transform_cdt

    inv = np.bitwise_not(free.astype("?")).astype(np.uint8)
    return distance_transform_cdt(inv, metric="taxicab").astype(np.float32)


class SuperGridRLRef:
    """``SuperGridRL`` (``super_grid_rl.py:18``) without pygame/rendering.

    ``positions`` (reset): optional [(x, y), ...] start cells instead of the
    NumPy RNG draw (used to replay device-drawn cells)."""

    def __init__(self, train_set, env_config, test_set=None):  # :27-72
        self._train_gridlis = train_set
        self._test_gridlis = test_set
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
        self.a_prev = None
        self.reset(False, False)
        self.a_inv = {2: 3, 3: 2, 0: 1, 1: 0}
        state = self.get_state()
        self._obs_dim = state[0].shape
        self._num_actions = 4 ** self._numrobot

    # ------------------------------------------------------------------
    def step(self, action):  # :74-225
        done = False
        if action is None or (not isinstance(action, (list, np.ndarray)) and action == -1):
            done = True
            reward = 0
        else:
            if type(action) != list:
                ulis = np.zeros((self._numrobot,))
                for i in range(self._numrobot):
                    ulis[i] = action % 4
                    action = action // 4
            else:
                ulis = action
            reward = np.zeros((self._numrobot,))
            pq = PriorityQueue()
            for i in range(self._numrobot):
                pq.put((self._xinds[i] + self._yinds[i] * self._gridwidth, i))
            r2c = np.zeros((self._numrobot,), dtype=int)
            if self._dist_r:
                distance_map = self.get_distance_map()
            for i in range(len(ulis)):
                u = ulis[i]
                z = pq.get()[1] if self._use_scanning else i
                r2c[z] = i
                x, y = self._xinds[z], self._yinds[z]
                if u == 0:
                    x = x - 1
                elif u == 1:
                    x = x + 1
                elif u == 2:
                    y = y + 1
                elif u == 3:
                    y = y - 1
                else:
                    continue
                if self.isInBounds(x, y) and not self.isOccupied(x, y):
                    self._xinds[z], self._yinds[z] = x, y
                    if self._dist_r:
                        reward[i] += distance_map[x, y]
                else:
                    reward[i] -= self._collision_penalty
            r = self._senseradius
            for i in range(self._numrobot):  # :177-201
                x, y = self._xinds[i], self._yinds[i]
                for j in range(x - r, x + r + 1):
                    for k in range(y - r, y + r + 1):
                        if not self.isInBounds(j, k):
                            continue
                        g = self._grid[j][k]
                        if g >= 0 and self._free[j][k] == 1:
                            reward[r2c[i]] += g
                            self._free[j][k] = 0
                        elif g >= 0 and self._free[j][k] == 0:
                            reward[r2c[i]] -= self._free_penalty
                        elif g < 0 and self._observed_obstacles[j][k] == 0:
                            self._observed_obstacles[j][k] = 1
            a = action
            if hasattr(a, "item") and not isinstance(a, (int, np.integer)):
                a = a.item()
            reward += self.motion_penalty(a)
            self.a_prev = a
            self._currstep += 1
            reward = np.sum(reward)
            if min(self._done_thresh, 1) <= self.percent_covered():
                reward += self._terminal_reward
        state = self.get_state()
        if done is False:
            done = self.done()
        return state, reward, done

    def motion_penalty(self, a):  # :227-243
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
        for a, b in zip(self._xinds, self._yinds):
            if a == x and b == y:
                return True
        return False

    def get_distance_map(self):  # :281-303
        d = l1_distance_to_uncovered(self._free)
        if np.max(d) > 0:
            d = d / np.max(d)
        return 1 - d

    def get_state(self):  # :305-317
        distance_map = self.get_distance_map()
        arrays = np.array(self.get_pos_image() + [self._observed_obstacles, self._free, distance_map])
        return np.stack(arrays, axis=0), self._currstep

    def get_pos_image(self):  # :319-341
        if self._use_scanning:
            ret = np.zeros((self._gridwidth, self._gridlen))
            for i, j in zip(self._xinds, self._yinds):
                ret[i, j] = 1
            return [ret]
        out = []
        for i, j in zip(self._xinds, self._yinds):
            layer = np.zeros((self._gridwidth, self._gridlen))
            layer[i, j] = 1
            out.append(layer)
        return out

    def reset(self, testing, ind, positions=None):  # :343-399
        if testing and self._test_gridlis is not None:
            self._grid = self._test_gridlis[ind]
        else:
            self._grid = self._train_gridlis[np.random.randint(len(self._train_gridlis))]
        self._gridwidth, self._gridlen = self._grid.shape[0], self._grid.shape[1]
        self._currstep = 0
        self._xinds = np.zeros(self._numrobot, dtype=int)
        self._yinds = np.zeros(self._numrobot, dtype=int)
        if positions is not None:
            for c, (x, y) in enumerate(positions):
                self._xinds[c], self._yinds[c] = int(x), int(y)
        else:
            seen = {}
            count = 0
            while count != self._numrobot:
                x = np.random.randint(self._gridwidth)
                y = np.random.randint(self._gridlen)
                if self._grid[x][y] >= 0 and (x, y) not in seen:
                    seen[(x, y)] = 1
                    self._xinds[count], self._yinds[count] = x, y
                    count += 1
        self._observed_obstacles = np.zeros((self._gridwidth, self._gridlen))
        self._free = np.ones((self._gridwidth, self._gridlen))
        self._currstep = 0
        return self.get_state(), self._grid

    def done(self):  # :401-414
        if min(self._done_thresh, 1) <= self.percent_covered():
            self._done_thresh += self._done_incr
            return True
        return False

    def percent_covered(self):  # :416-421
        return np.count_nonzero(self._free < 1) / np.count_nonzero(self._grid > 0)

    # ------------------------------------------------------------------
    def snapshot(self):
        """State for golden fixtures / parity checks."""
        return dict(x=self._xinds.copy(), y=self._yinds.copy(),
                    free=self._free.copy(), obst=self._observed_obstacles.copy(),
                    currstep=self._currstep, done_thresh=float(self._done_thresh),
                    a_prev=-1 if self.a_prev is None else int(self.a_prev))
