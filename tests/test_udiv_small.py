"""render.hip UDivSmall: floor(y / d) for y < 2^21 as fl(fl(y + 1/2) * rcp(d)), v_rcp_f32 within 1 ulp of
1/d. Restated in numpy float32 with the reciprocal at its correctly rounded value and one ulp either
side (the hardware's error bound), over every y < 2^21 for divisors the shading kernel's row mapping
meets (band rows, tile-row cycles) and a spread of others -- the exactness claim in its comment."""
from __future__ import annotations

import numpy as np
import pytest

Y = np.arange(1 << 21, dtype=np.uint32)
YF = Y.astype(np.float32) + np.float32(0.5)  # exact: y < 2^23


@pytest.mark.parametrize("d", [1, 2, 3, 7, 8, 15, 16, 17, 135, 264, 270, 540, 816, 1079, 1080, 2160, 4095,
                               65535, 65536, 1 << 20, (1 << 21) - 1, 3 * 5 * 7 * 11 * 13])
def test_udiv_small_exact(d):
    r = np.float32(1.0) / np.float32(d)  # correctly rounded
    want = Y // np.uint32(d)
    for rr in (np.nextafter(r, np.float32(0)), r, np.nextafter(r, np.float32(np.inf))):
        got = (YF * np.float32(rr)).astype(np.uint32)  # one rounding of the product, then truncation
        assert np.array_equal(got, want), (d, rr)
