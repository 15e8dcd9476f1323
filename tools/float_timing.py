"""Device time per inference (graph replay) of the fp16-weight models next to
their int8 twins.  Diagnostic."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from band_amd import DeviceFlag, HipModel, HipModelExecutor, SubgraphKey, tflite_synth as S  # noqa: E402

for mid, (name, buf) in enumerate([("mobilenet_v2_fp16", S.mobilenet_v2(np.float16)),
                                   ("ssd_mobilenet_v2_fp16", S.ssd_mobilenet_v2(np.float16)),
                                   ("mobilenet_v2_int8", S.mobilenet_v2(np.int8))]):
    f = tempfile.NamedTemporaryFile(suffix=".tflite", delete=False)
    f.write(buf)
    f.close()
    m = HipModel(mid)
    assert m.FromPath(f.name).ok()
    ex = HipModelExecutor(mid, 1, DeviceFlag.kGPU)
    assert ex.PrepareSubgraph(m).ok()
    key = SubgraphKey(mid, 1)
    us = ex.TimeSubgraph(key, iters=50)
    top = sorted(ex.ProfileSubgraph(key, iters=10), key=lambda r: -r["ms"])[:5]
    print("%-24s %8.1f us  top: %s" % (name, us, ", ".join("%s %.1fus" % (r["kernel"], r["ms"] * 1e3) for r in top)))
    os.unlink(f.name)
