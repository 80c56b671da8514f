"""Product counterpart of the reference utils.py (quaternion_to_euler, utils.py:3-21)."""
import numpy as np


def quaternion_to_euler(quat):
    """(w, x, y, z) -> (roll, pitch, yaw).  Pitch is arcsin(2(wy - zx)) WITHOUT clamping, so it
    is NaN when |2(wy - zx)| > 1, exactly as the reference (utils.py:13-14)."""
    w, x, y, z = quat
    roll = np.arctan2(2 * (w * x + y * z), 1 - 2 * (x * x + y * y))
    with np.errstate(invalid="ignore"):
        pitch = np.arcsin(2 * (w * y - z * x))
    yaw = np.arctan2(2 * (w * z + x * y), 1 - 2 * (y * y + z * z))
    return roll, pitch, yaw
