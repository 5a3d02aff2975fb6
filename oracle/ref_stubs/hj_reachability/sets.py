import numpy as _np


class Box(object):
    """Restated ``hj.sets.Box``: extreme_point = where(direction < 0, lo, hi) (float32)."""

    def __init__(self, lo, hi):
        self.lo = _np.asarray(lo)
        self.hi = _np.asarray(hi)

    def extreme_point(self, direction):
        d = _np.asarray(direction)
        return _np.where(d < 0, self.lo.astype(_np.float32),
                         self.hi.astype(_np.float32)).astype(_np.float32)
