#!/usr/bin/env python3
"""Phase breakdown (share of all wave cycles) of a RT_STAMPS timeline dump:
  tl_breakdown.py FILE NWAVES"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16)[: int(sys.argv[2])].astype(np.int64)
a = a[a[:, 1] > 0]
tot = a[:, 7].sum()
print("waves %d  total wave cycles %.3g" % (len(a), tot))
for nm, i in [("closest sweeps", 12), ("shadow queries", 13), ("  bvh walks", 10), ("  bound", 3), ("  cull", 4),
              ("  candidate tests", 5), ("shading", 6), ("light setup", 11)]:
    print("%-18s %.3g %5.1f%%" % (nm, a[:, i].sum(), 100 * a[:, i].sum() / tot))
