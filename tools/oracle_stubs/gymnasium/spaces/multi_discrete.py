import numpy as np


class MultiDiscrete:
    def __init__(self, nvec, dtype=np.int64):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
