"""Sensor configuration objects of the reference (``Environments/Sensors``).

On this framework the measurement itself runs inside the HIP step kernel;
these classes hold the sensor parameters and, for the lidar, the per-beam
increment table the kernel marches with.  The table is computed on the host
with NumPy scalar operations in exactly the order ``lidar.py:38-48`` uses, so
the device march starts from the same float64 bits as the reference.
"""
from __future__ import annotations

import weakref

import numpy as np


def beam_angles(num_lasers: int) -> np.ndarray:
    """``lidar.py:14``: equally spaced, endpoint excluded."""
    return np.linspace(0, 2 * np.pi, num=num_lasers, endpoint=False)


def beam_increments(thetalist) -> np.ndarray:
    """[B, 3] float64 rows (xinc, yinc, distinc) per beam (``lidar.py:38-48``)."""
    rows = np.empty((len(thetalist), 3), dtype=np.float64)
    for i, th in enumerate(thetalist):
        cx = np.cos(th)
        cy = np.sin(th)
        norm = max(abs(cx), abs(cy))
        cx /= norm
        cy /= norm
        rows[i] = (cx, cy, np.sqrt(cx ** 2 + cy ** 2))
    return rows


class Sensor:
    """``Environments/Sensors/Sensor.py``: parameter holder."""

    sensor_type = None

    def __init__(self):
        self._listeners = []     # weakref.WeakMethod of each device env's uploader

    def add_listener(self, bound_method):
        """Weakly register ``bound_method(sensor)``: a shared sensor must not
        keep the device envs built on it alive."""
        self._listeners.append(weakref.WeakMethod(bound_method))

    def remove_listener(self, bound_method):
        self._listeners = [w for w in self._listeners if w() is not None and w() != bound_method]

    def _changed(self):
        """Call every live listener (all of them, even after one fails: a
        shared sensor must not leave its envs on different tables), prune the
        dead ones, then re-raise the first failure."""
        live, err = [], None
        for w in self._listeners:
            fn = w()
            if fn is None:
                continue
            live.append(w)
            try:
                fn(self)
            except Exception as e:  # noqa: BLE001 -- re-raised below
                err = err or e
        self._listeners = live
        if err is not None:
            raise err


class LidarSensor(Sensor):
    """``lidar.py:5-14``.  ``allow_even`` lifts the odd-count assert (the
    batched configs use 360 beams)."""

    sensor_type = "lidar"

    def __init__(self, sensor_config, allow_even=False):
        super().__init__()
        self._num_lasers = int(sensor_config["num_lasers"])
        self._max_range = sensor_config["range"]
        if not allow_even:
            assert self._num_lasers % 2 == 1, "odd number of lasers needed"
        self._thetalist = beam_angles(self._num_lasers)

    def set_thetalist(self, thetalist):
        """Replace the beam angles (any count); pushes the new table to every
        device env built on this sensor.  If a device env rejects the table
        (mc_set_beam_table validates before it changes anything), the old
        angles are restored and pushed to every env again, then the error is
        raised: sensor, configs and devices never disagree."""
        old = (self._thetalist, self._num_lasers)
        self._thetalist = np.asarray(thetalist, dtype=np.float64)
        self._num_lasers = len(self._thetalist)
        try:
            self._changed()
        except Exception:
            self._thetalist, self._num_lasers = old
            self._changed()
            raise

    def table(self) -> np.ndarray:
        return beam_increments(self._thetalist)

    def window_half(self) -> int:
        r = float(self._max_range)
        return int(np.ceil(r)) if r > 0 else 0


class SquareSensor(Sensor):
    """``squaresensor.py:4-13``."""

    sensor_type = "square_sensor"

    def __init__(self, sensor_config):
        super().__init__()
        self._radius = int(sensor_config["range"])

    def window_half(self) -> int:
        return self._radius


def make_sensor(env_config):
    kind = env_config["sensor_type"]
    if kind == "lidar":
        return LidarSensor(env_config["sensor_config"],
                           allow_even=bool(env_config.get("allow_even_beams", False)))
    if kind == "square_sensor":
        return SquareSensor(env_config["sensor_config"])
    raise ValueError(f"unknown sensor_type {kind!r}")
