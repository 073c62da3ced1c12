"""Physical constants used by the FD waveform path.

The values are FastEMRIWaveforms' (`few.utils.constants`), which the reference imports with
`from few.utils.constants import *` (check_mode_by_mode.py:46, emri_pe.py:63,
Tutorial_FD_construction_single_mode.ipynb:25-45). MTSUN_SI is pinned by the known answer
printed at Tutorial_FD_construction_single_mode.ipynb:301 (see tests/test_physics_standins.py).
"""

import math

MTSUN_SI = 4.925491025543576e-06      # G M_sun / c^3 [s]
MRSUN_SI = 1476.6250614046494         # G M_sun / c^2 [m]
Gpc = 3.0856775814913673e25           # [m]
YRSID_SI = 31558149.763545603         # sidereal year [s]
PI = math.pi

__all__ = ["MTSUN_SI", "MRSUN_SI", "Gpc", "YRSID_SI", "PI"]
