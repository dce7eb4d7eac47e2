"""RawRead mirror (reference: misc/raw_read.py:18-45): int8 band-sequential raw rasters."""

import numpy as np


class RawRead():
    '''
    read raw image and convert it to numpy array
    '''

    def __init__(self):
        pass

    @staticmethod
    def _read8(filename, xdata, ydata, band):
        """c[band, y, x] from an int8 raw file (np.fromfile, memory-light)."""
        c = np.fromfile(filename, dtype=np.int8, count=xdata * ydata * band).reshape(band, ydata, xdata)
        return c

    @classmethod
    def read(self, path, size=(6000, 6000), rate=1):
        '''
        read image: int8 * rate, wrapped to uint8 (as the reference's astype)
        '''
        return (self._read8(path, size[0], size[1], 1) * rate)[0].astype(np.uint8)
