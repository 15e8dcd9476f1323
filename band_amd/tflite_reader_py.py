"""Small .tflite reader used by the synthesiser's uint8->int8 conversion.

Returns plain dicts and re-materialises builtin options as writer Tables so
a model can be rewritten.  (The backend's own reader is C++:
band_amd/csrc/backend/hip/tflite_reader.cc.)
"""
import struct

import numpy as np

from . import tflite_synth as S

_NP = {0: np.float32, 2: np.int32, 3: np.uint8, 4: np.int64, 9: np.int8, 7: np.int16}

# BuiltinOptions union index -> [(slot, fmt)], fmt 'vi' = vector<int>
OPTION_FIELDS = {
    1: [(0, "b"), (1, "i"), (2, "i"), (3, "b"), (4, "i"), (5, "i")],            # Conv2D
    2: [(0, "b"), (1, "i"), (2, "i"), (3, "i"), (4, "b"), (5, "i"), (6, "i")],  # DepthwiseConv2D
    5: [(0, "b"), (1, "i"), (2, "i"), (3, "i"), (4, "i"), (5, "b")],            # Pool2D
    8: [(0, "b"), (1, "b"), (2, "B"), (3, "B")],                                # FullyConnected
    9: [(0, "f")],                                                              # Softmax
    10: [(0, "i"), (1, "b")],                                                   # Concatenation
    11: [(0, "b"), (1, "B")],                                                   # Add
    17: [(0, "vi")],                                                            # Reshape
    21: [(0, "b")],                                                             # Mul
    28: [(0, "b"), (1, "B")],                                                   # Sub
}


class _T:
    def __init__(self, buf, pos):
        self.b, self.p = buf, pos
        self.vt = pos - struct.unpack_from("<i", buf, pos)[0]
        self.vl = struct.unpack_from("<H", buf, self.vt)[0]

    def off(self, s):
        o = 4 + 2 * s
        return 0 if o >= self.vl else struct.unpack_from("<H", self.b, self.vt + o)[0]

    def sc(self, s, fmt, d=0):
        o = self.off(s)
        return d if not o else struct.unpack_from("<" + fmt, self.b, self.p + o)[0]

    def ref(self, s):
        o = self.off(s)
        if not o:
            return None
        return self.p + o + struct.unpack_from("<I", self.b, self.p + o)[0]

    def tab(self, s):
        r = self.ref(s)
        return None if r is None else _T(self.b, r)

    def vec(self, s, fmt):
        r = self.ref(s)
        if r is None:
            return None
        n = struct.unpack_from("<I", self.b, r)[0]
        return np.frombuffer(self.b, dtype="<" + fmt, count=n, offset=r + 4)

    def tabs(self, s):
        r = self.ref(s)
        if r is None:
            return []
        n = struct.unpack_from("<I", self.b, r)[0]
        return [_T(self.b, r + 4 + 4 * i + struct.unpack_from("<I", self.b, r + 4 + 4 * i)[0]) for i in range(n)]

    def str(self, s):
        r = self.ref(s)
        if r is None:
            return ""
        n = struct.unpack_from("<I", self.b, r)[0]
        return bytes(self.b[r + 4:r + 4 + n]).decode("utf-8", "replace")


def _options(t, kind):
    if t is None or kind not in OPTION_FIELDS:
        return None
    out = S.Table()
    for slot, fmt in OPTION_FIELDS[kind]:
        if not t.off(slot):
            continue
        if fmt == "vi":
            out.set(slot, "o", S.Vec("i", [int(v) for v in t.vec(slot, "i4")]))
        else:
            out.set(slot, fmt, t.sc(slot, fmt))
    return out


def read(data):
    buf = bytes(data)
    root = _T(buf, struct.unpack_from("<I", buf, 0)[0])
    codes = [max(oc.sc(0, "b"), oc.sc(3, "i")) for oc in root.tabs(1)]
    bufs = root.tabs(4)
    sg = root.tabs(2)[0]
    tensors = []
    for t in sg.tabs(0):
        shape = [int(v) for v in (t.vec(0, "i4") if t.vec(0, "i4") is not None else [])]
        typ = t.sc(1, "b")
        q = t.tab(4)
        scale = zp = None
        qdim = 0
        if q is not None and q.vec(2, "f4") is not None and len(q.vec(2, "f4")):
            scale = [float(v) for v in q.vec(2, "f4")]
            z = q.vec(3, "i8")
            zp = [int(v) for v in z] if z is not None else [0] * len(scale)
            qdim = q.sc(6, "i")
        bi = t.sc(2, "I")
        data_ = None
        if 0 < bi < len(bufs):
            raw = bufs[bi].vec(0, "u1")
            if raw is not None and len(raw):
                data_ = np.frombuffer(bytes(raw), dtype=_NP[typ]).reshape(shape)
        tensors.append(dict(name=t.str(3), shape=shape, type=typ, scale=scale, zero_point=zp, qdim=qdim, data=data_))
    ops = []
    for o in sg.tabs(3):
        kind = o.sc(3, "B")
        ops.append(dict(builtin=codes[o.sc(0, "I")], inputs=[int(v) for v in o.vec(1, "i4")],
                        outputs=[int(v) for v in o.vec(2, "i4")], options_type=kind if kind in OPTION_FIELDS else 0,
                        options=_options(o.tab(4), kind)))
    return dict(description=root.str(3), tensors=tensors, ops=ops,
                inputs=[int(v) for v in sg.vec(1, "i4")], outputs=[int(v) for v in sg.vec(2, "i4")])
