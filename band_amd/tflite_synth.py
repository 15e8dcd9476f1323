"""Write TFLite schema-v3 flatbuffers and synthesise the BASELINE models.

Five of the six BASELINE.json models are not in the reference's fixtures
(band/test/data/ holds only mobilenet_v2_1.0_224_quant, retinaface, ICN and
magenta), and there is no network, so bench and tests build
them here as .tflite files with the same operator set a TFLite converter
emits.  Weights are synthetic (seeded) unless converted from a real model.

Nothing here is on the hot path: it produces the *input* of IModel::FromPath
(band/backend/tfl/model.cc:25-39).  The writer is dependency-free (no
flatbuffers package): tables are laid out front-to-back with each child
written after its parent so every uoffset is forward, as the format needs.
"""
import struct

import numpy as np

# schema enums
T_FLOAT32, T_FLOAT16, T_INT32, T_UINT8, T_INT8 = 0, 1, 2, 3, 9
NP_TO_SCHEMA = {np.dtype(np.float32): T_FLOAT32, np.dtype(np.float16): T_FLOAT16, np.dtype(np.int32): T_INT32,
                np.dtype(np.uint8): T_UINT8, np.dtype(np.int8): T_INT8}
ACT = {"NONE": 0, "RELU": 1, "RELU_N1_TO_1": 2, "RELU6": 3}
OPC = dict(ADD=0, AVERAGE_POOL_2D=1, CONCATENATION=2, CONV_2D=3, DEPTHWISE_CONV_2D=4,
           FULLY_CONNECTED=9, LOGISTIC=14, MAX_POOL_2D=17, MUL=18, RESHAPE=22,
           RESIZE_BILINEAR=23, SOFTMAX=25, CUSTOM=32, PAD=34, SUB=41, QUANTIZE=114,
           DEQUANTIZE=6, RELU=19, RELU_N1_TO_1=20, RELU6=21, PADV2=60, RESIZE_NEAREST_NEIGHBOR=97,
           TRANSPOSE_CONV=67)
# BuiltinOptions union indices
OPT = dict(Conv2DOptions=1, DepthwiseConv2DOptions=2, Pool2DOptions=5, FullyConnectedOptions=8,
           SoftmaxOptions=9, ConcatenationOptions=10, AddOptions=11, ReshapeOptions=17,
           ResizeBilinearOptions=15, MulOptions=21, PadOptions=22, SubOptions=28,
           DequantizeOptions=38, PadV2Options=43, TransposeConvOptions=49, ResizeNearestNeighborOptions=74,
           QuantizeOptions=89)


# ---------------------------------------------------------------------------
# FlexBuffers map (the encoding of TFLite custom options)
# ---------------------------------------------------------------------------
FBT_INT, FBT_FLOAT, FBT_MAP, FBT_BOOL = 1, 3, 9, 26


def flexbuffer_map(values):
    """A FlexBuffers map of scalars: sorted keys, 8-byte elements.  Layout:
    key strings, the typed key vector, [keys offset, keys width, size],
    elements, one packed type byte per element, then the root (offset, type,
    width)."""
    buf = bytearray()

    def align(n):
        while len(buf) % n:
            buf.append(0)

    keys = sorted(values)
    key_pos = []
    for k in keys:
        key_pos.append(len(buf))
        buf += k.encode() + b"\0"
    align(8)
    buf += struct.pack("<Q", len(keys))
    keys_start = len(buf)
    for kp in key_pos:
        buf += struct.pack("<Q", len(buf) - kp)
    align(8)
    buf += struct.pack("<Q", len(buf) - keys_start)  # keys vector, relative
    buf += struct.pack("<Q", 8)                      # keys element width
    buf += struct.pack("<Q", len(keys))
    map_start = len(buf)
    types = []
    for k in keys:
        v = values[k]
        if isinstance(v, bool):
            buf += struct.pack("<Q", int(v))
            types.append(FBT_BOOL << 2 | 3)
        elif isinstance(v, (int, np.integer)):
            buf += struct.pack("<q", int(v))
            types.append(FBT_INT << 2 | 3)
        else:
            buf += struct.pack("<d", float(v))
            types.append(FBT_FLOAT << 2 | 3)
    buf += bytes(types)
    align(8)
    buf += struct.pack("<Q", len(buf) - map_start)
    buf += bytes([FBT_MAP << 2 | 3, 8])
    return bytes(buf)


# ---------------------------------------------------------------------------
# minimal flatbuffer serializer
# ---------------------------------------------------------------------------
class Table:
    """fields: {slot: (fmt, value)} for scalars, {slot: ('o', obj)} for children."""

    def __init__(self, **kw):
        self.fields = {}

    def set(self, slot, fmt, value):
        self.fields[slot] = (fmt, value)
        return self


class Vec:
    def __init__(self, fmt, values, align=4):
        self.fmt = fmt
        self.values = values
        self.align = align


class VecT:
    def __init__(self, items):
        self.items = items


class Str:
    def __init__(self, s):
        self.s = s.encode() if isinstance(s, str) else bytes(s)


class _Writer:
    def __init__(self):
        self.buf = bytearray()

    def pad_to(self, n, extra=0):
        while (len(self.buf) + extra) % n:
            self.buf.append(0)

    def write(self, obj):
        if isinstance(obj, Table):
            return self._table(obj)
        if isinstance(obj, Vec):
            return self._vec(obj)
        if isinstance(obj, VecT):
            return self._vect(obj)
        if isinstance(obj, Str):
            self.pad_to(4)
            pos = len(self.buf)
            self.buf += struct.pack("<I", len(obj.s)) + obj.s + b"\0"
            return pos
        raise TypeError(obj)

    def _vec(self, v):
        if isinstance(v.values, (bytes, bytearray, np.ndarray)):
            raw = bytes(np.ascontiguousarray(v.values).tobytes()) if isinstance(v.values, np.ndarray) else bytes(v.values)
            n = len(raw) // struct.calcsize("<" + v.fmt)
        else:
            raw = b"".join(struct.pack("<" + v.fmt, x) for x in v.values)
            n = len(v.values)
        self.pad_to(max(v.align, 4), extra=4)
        pos = len(self.buf)
        self.buf += struct.pack("<I", n) + raw
        return pos

    def _vect(self, v):
        self.pad_to(4)
        pos = len(self.buf)
        self.buf += struct.pack("<I", len(v.items))
        slots = []
        for _ in v.items:
            slots.append(len(self.buf))
            self.buf += b"\0\0\0\0"
        for slot, item in zip(slots, v.items):
            cpos = self.write(item)
            struct.pack_into("<I", self.buf, slot, cpos - slot)
        return pos

    def _table(self, t):
        slots = sorted(t.fields)
        nslots = (max(slots) + 1) if slots else 0
        # field layout inside the table: scalars by size (desc), then offsets
        items = []
        for s in slots:
            fmt, val = t.fields[s]
            size = 4 if fmt == "o" else struct.calcsize("<" + fmt)
            items.append((size, s, fmt, val))
        items.sort(key=lambda x: -x[0])
        layout = {}
        off = 4  # soffset to vtable
        for size, s, fmt, val in items:
            off = (off + size - 1) // size * size
            layout[s] = off
            off += size
        tsize = off
        vt = struct.pack("<HH", 4 + 2 * nslots, tsize) + b"".join(
            struct.pack("<H", layout.get(i, 0)) for i in range(nslots))
        self.pad_to(2)
        vt_pos = len(self.buf)
        self.buf += vt
        self.pad_to(8)
        tpos = len(self.buf)
        self.buf += bytearray(tsize)
        struct.pack_into("<i", self.buf, tpos, tpos - vt_pos)
        children = []
        for size, s, fmt, val in items:
            p = tpos + layout[s]
            if fmt == "o":
                children.append((p, val))
            else:
                struct.pack_into("<" + fmt, self.buf, p, val)
        for p, child in children:
            cpos = self.write(child)
            struct.pack_into("<I", self.buf, p, cpos - p)
        return tpos


def serialize(root):
    w = _Writer()
    w.buf += b"\0\0\0\0TFL3"
    rpos = w.write(root)
    struct.pack_into("<I", w.buf, 0, rpos)
    return bytes(w.buf)


# ---------------------------------------------------------------------------
# model description -> flatbuffer
# ---------------------------------------------------------------------------
class ModelBuilder:
    """Collects tensors / buffers / operators of one subgraph."""

    def __init__(self, description="band_amd synthetic"):
        self.tensors = []   # dicts
        self.buffers = [b""]  # buffer 0 is the empty sentinel
        self.ops = []
        self.opcodes = []   # (builtin, custom)
        self.inputs = []
        self.outputs = []
        self.description = description

    def tensor(self, name, shape, dtype, scale=None, zero_point=None, qdim=0, data=None):
        buf = 0
        if data is not None:
            arr = np.ascontiguousarray(np.asarray(data, dtype=dtype).reshape(shape))
            self.buffers.append(arr.tobytes())
            buf = len(self.buffers) - 1
        self.tensors.append(dict(name=name, shape=list(shape), type=NP_TO_SCHEMA[np.dtype(dtype)],
                                 buffer=buf, scale=scale, zero_point=zero_point, qdim=qdim))
        return len(self.tensors) - 1

    def op(self, builtin, inputs, outputs, options_type=0, options=None, custom=None, custom_options=None):
        key = (OPC[builtin] if isinstance(builtin, str) else builtin, custom)
        if key not in self.opcodes:
            self.opcodes.append(key)
        self.ops.append(dict(opcode=self.opcodes.index(key), inputs=list(inputs), outputs=list(outputs),
                             options_type=options_type, options=options, custom_options=custom_options))
        return len(self.ops) - 1

    def build(self):
        tens = []
        for t in self.tensors:
            tt = Table().set(0, "o", Vec("i", t["shape"])).set(1, "b", t["type"]).set(2, "I", t["buffer"])
            tt.set(3, "o", Str(t["name"]))
            if t["scale"] is not None:
                sc = [float(x) for x in np.atleast_1d(t["scale"])]
                zp = [int(x) for x in np.atleast_1d(t["zero_point"] if t["zero_point"] is not None else 0)]
                if len(zp) != len(sc):
                    zp = zp * len(sc) if len(zp) == 1 else zp
                q = Table().set(2, "o", Vec("f", sc)).set(3, "o", Vec("q", zp)).set(6, "i", int(t["qdim"]))
                tt.set(4, "o", q)
            tens.append(tt)
        ops = []
        for o in self.ops:
            ot = Table().set(0, "I", o["opcode"]).set(1, "o", Vec("i", o["inputs"])).set(2, "o", Vec("i", o["outputs"]))
            if o["options_type"]:
                ot.set(3, "B", o["options_type"]).set(4, "o", o["options"])
            if o.get("custom_options") is not None:
                ot.set(5, "o", Vec("B", o["custom_options"]))  # custom_options_format FLEXBUFFERS (0)
            ops.append(ot)
        sg = (Table().set(0, "o", VecT(tens)).set(1, "o", Vec("i", self.inputs))
              .set(2, "o", Vec("i", self.outputs)).set(3, "o", VecT(ops)).set(4, "o", Str("main")))
        codes = []
        for b, c in self.opcodes:
            oc = Table().set(0, "b", min(b, 127)).set(2, "i", 1).set(3, "i", b)
            if c:
                oc.set(1, "o", Str(c))
            codes.append(oc)
        bufs = [Table() if not b else Table().set(0, "o", Vec("B", b, align=16)) for b in self.buffers]
        root = (Table().set(0, "I", 3).set(1, "o", VecT(codes)).set(2, "o", VecT([sg]))
                .set(3, "o", Str(self.description)).set(4, "o", VecT(bufs)))
        return serialize(root)


def conv_options(padding, stride, act, dilation=1):
    return (Table().set(0, "b", 0 if padding == "SAME" else 1).set(1, "i", stride).set(2, "i", stride)
            .set(3, "b", ACT[act]).set(4, "i", dilation).set(5, "i", dilation))


def dw_options(padding, stride, act, dm=1, dilation=1):
    return (Table().set(0, "b", 0 if padding == "SAME" else 1).set(1, "i", stride).set(2, "i", stride)
            .set(3, "i", dm).set(4, "b", ACT[act]).set(5, "i", dilation).set(6, "i", dilation))


def pool_options(padding, stride, filt, act="NONE"):
    return (Table().set(0, "b", 0 if padding == "SAME" else 1).set(1, "i", stride).set(2, "i", stride)
            .set(3, "i", filt[1]).set(4, "i", filt[0]).set(5, "b", ACT[act]))


def act_options(act="NONE"):
    return Table().set(0, "b", ACT[act])


# ---------------------------------------------------------------------------
# quantised graph construction with synthetic (seeded) weights
# ---------------------------------------------------------------------------
class QGraph:
    """Builds an int8 (per-channel) or uint8 (per-tensor) NHWC graph.

    Scales mimic converter output (RELU6 tensors at 6/255) and filter scales
    are chosen per layer so activations stay spread over the 8-bit range
    instead of collapsing or saturating, which keeps bit-exact checks
    meaningful (BASELINE.md's log-uniform [1e-3, 2e-2] filter scales collapse
    a 65-op network to constants within a few layers).
    """

    def __init__(self, dtype=np.int8, seed=0, name="model"):
        self.dtype = np.dtype(dtype)
        self.rng = np.random.default_rng(seed)
        self.mb = ModelBuilder(name)
        self.n = 0
        self.meta = {}  # tensor -> (shape, scale, zp)
        self.fshape = {}  # float32 tensor -> shape

    def _name(self, kind):
        self.n += 1
        return "%s_%d" % (kind, self.n)

    def _act_zp(self):
        return int(self.rng.integers(-20, 21)) if self.dtype == np.int8 else int(self.rng.integers(108, 149))

    def act_tensor(self, shape, scale, zp, kind="act"):
        t = self.mb.tensor(self._name(kind), shape, self.dtype, scale=[scale], zero_point=[zp])
        self.meta[t] = (list(shape), scale, zp)
        return t

    def input(self, shape, scale=0.0078125, zp=None):
        zp = (0 if self.dtype == np.int8 else 128) if zp is None else zp
        t = self.act_tensor(shape, scale, zp, "input")
        self.mb.inputs.append(t)
        return t

    def output(self, t):
        self.mb.outputs.append(t)

    def _out_q(self, act, s_in):
        """Output (scale, zero point) the way converted models look: RELU6/RELU
        outputs cover [0, 6] (scale 6/255, zero point at the range bottom);
        linear outputs keep the input scale around a small zero point."""
        if act in ("RELU6", "RELU"):
            return 6.0 / 255.0, (-128 if self.dtype == np.int8 else 0)
        return float(s_in), self._act_zp()

    def _weights(self, shape, out_c, qdim, s_in, s_out, K):
        # filter scale chosen so sum_k x*w lands ~40 output LSBs wide
        # (|x - zp| ~ 45 LSB, |w| ~ 73 LSB), jittered per channel
        base = 40.0 * s_out / (s_in * np.sqrt(K) * 45.0 * 73.0)
        if self.dtype == np.int8:
            w = self.rng.integers(-127, 128, size=shape).astype(np.int8)
            ws = (base * np.exp(self.rng.uniform(-0.4, 0.4, size=out_c))).astype(np.float32)
            wt = self.mb.tensor(self._name("weights"), shape, np.int8, scale=ws, zero_point=[0] * out_c,
                                qdim=qdim, data=w)
            return wt, ws
        w = self.rng.integers(0, 256, size=shape).astype(np.uint8)
        ws = np.array([base * np.exp(self.rng.uniform(-0.4, 0.4))], np.float32)
        wt = self.mb.tensor(self._name("weights"), shape, np.uint8, scale=ws,
                            zero_point=[int(self.rng.integers(125, 132))], data=w)
        return wt, ws

    def _bias(self, out_c, in_scale, ws, K):
        lim = max(1, int(np.sqrt(K) * 45 * 73 / 3))
        b = self.rng.integers(-lim, lim + 1, size=out_c).astype(np.int32)
        bs = (np.float32(in_scale) * (ws if len(ws) > 1 else np.repeat(ws, out_c))).astype(np.float32)
        return self.mb.tensor(self._name("bias"), [out_c], np.int32, scale=bs, zero_point=[0] * out_c, data=b)

    def conv(self, x, out_c, k=1, stride=1, act="RELU6", padding="SAME", dilation=1, out_scale=None,
             bias_offset_lsb=0):
        """CONV_2D; `out_scale` overrides the output scale and
        `bias_offset_lsb` shifts every output channel by that many output
        LSBs (a detection head's class prior)"""
        shp, s_in, _ = self.meta[x]
        b, h, w, c = shp
        s_out, zp = self._out_q(act, s_in)
        if out_scale is not None:
            s_out = float(out_scale)
        K = k * k * c
        wt, ws = self._weights([out_c, k, k, c], out_c, 0, s_in, s_out, K)
        bt = self._bias(out_c, s_in, ws, K)
        if bias_offset_lsb:
            bias = self.mb.tensors[bt]
            bufi = bias["buffer"]
            vals = np.frombuffer(self.mb.buffers[bufi], np.int32).copy()
            wsc = ws if len(ws) > 1 else np.repeat(ws, out_c)
            vals += np.round(bias_offset_lsb * s_out / (s_in * wsc.astype(np.float64))).astype(np.int32)
            self.mb.buffers[bufi] = vals.tobytes()
        eff = (k - 1) * dilation + 1
        oh = (h + stride - 1) // stride if padding == "SAME" else (h + stride - eff) // stride
        ow = (w + stride - 1) // stride if padding == "SAME" else (w + stride - eff) // stride
        y = self.act_tensor([b, oh, ow, out_c], s_out, zp)
        self.mb.op("CONV_2D", [x, wt, bt], [y], OPT["Conv2DOptions"], conv_options(padding, stride, act, dilation))
        return y

    def dwconv(self, x, k=3, stride=1, act="RELU6", padding="SAME", dm=1, dilation=1):
        shp, s_in, _ = self.meta[x]
        b, h, w, c = shp
        oc = c * dm
        s_out, zp = self._out_q(act, s_in)
        wt, ws = self._weights([1, k, k, oc], oc, 3, s_in, s_out, k * k)
        bt = self._bias(oc, s_in, ws, k * k)
        eff = (k - 1) * dilation + 1
        oh = (h + stride - 1) // stride if padding == "SAME" else (h + stride - eff) // stride
        ow = (w + stride - 1) // stride if padding == "SAME" else (w + stride - eff) // stride
        y = self.act_tensor([b, oh, ow, oc], s_out, zp)
        self.mb.op("DEPTHWISE_CONV_2D", [x, wt, bt], [y], OPT["DepthwiseConv2DOptions"],
                   dw_options(padding, stride, act, dm, dilation))
        return y

    def add(self, a, b, act="NONE"):
        shp, sa, _ = self.meta[a]
        _, sb, _ = self.meta[b]
        y = self.act_tensor(shp, float(max(sa, sb) * 1.4), self._act_zp())
        self.mb.op("ADD", [a, b], [y], OPT["AddOptions"], act_options(act))
        return y

    def avgpool(self, x, filt, stride=1, padding="VALID"):
        shp, s, z = self.meta[x]
        b, h, w, c = shp
        oh = (h + stride - filt[0]) // stride if padding == "VALID" else (h + stride - 1) // stride
        ow = (w + stride - filt[1]) // stride if padding == "VALID" else (w + stride - 1) // stride
        y = self.act_tensor([b, oh, ow, c], s, z)
        self.mb.op("AVERAGE_POOL_2D", [x], [y], OPT["Pool2DOptions"], pool_options(padding, stride, filt))
        return y

    def maxpool(self, x, filt, stride, padding="SAME"):
        shp, s, z = self.meta[x]
        b, h, w, c = shp
        oh = (h + stride - filt[0]) // stride if padding == "VALID" else (h + stride - 1) // stride
        ow = (w + stride - filt[1]) // stride if padding == "VALID" else (w + stride - 1) // stride
        y = self.act_tensor([b, oh, ow, c], s, z)
        self.mb.op("MAX_POOL_2D", [x], [y], OPT["Pool2DOptions"], pool_options(padding, stride, filt))
        return y

    def reshape(self, x, shape):
        _, s, z = self.meta[x]
        st = self.mb.tensor(self._name("shape"), [len(shape)], np.int32, data=np.array(shape, np.int32))
        y = self.act_tensor(list(shape), s, z)
        self.mb.op("RESHAPE", [x, st], [y], OPT["ReshapeOptions"], Table().set(0, "o", Vec("i", list(shape))))
        return y

    def fully_connected(self, x, units, act="NONE"):
        shp, s_in, _ = self.meta[x]
        depth = shp[-1]
        rows = int(np.prod(shp)) // depth
        w = (self.rng.integers(-127, 128, size=(units, depth)).astype(np.int8) if self.dtype == np.int8
             else self.rng.integers(0, 256, size=(units, depth)).astype(np.uint8))
        ws = np.array([np.exp(self.rng.uniform(np.log(1e-3), np.log(2e-2)))], np.float32)
        wzp = 0 if self.dtype == np.int8 else int(self.rng.integers(125, 132))
        s_out, zp = self._out_q(act, s_in)
        ws = np.array([40.0 * s_out / (s_in * np.sqrt(depth) * 45.0 * 73.0)], np.float32)
        wt = self.mb.tensor(self._name("fc_weights"), [units, depth], self.dtype, scale=ws, zero_point=[wzp], data=w)
        bt = self._bias(units, s_in, ws, depth)
        y = self.act_tensor([rows, units], s_out, zp)
        self.mb.op("FULLY_CONNECTED", [x, wt, bt], [y], OPT["FullyConnectedOptions"], act_options(act))
        return y

    # --- glue ops ------------------------------------------------------------
    def _like(self, x, shape=None, scale=None, zp=None):
        shp, s, z = self.meta[x]
        return self.act_tensor(list(shape if shape is not None else shp), s if scale is None else scale,
                               z if zp is None else zp)

    def quantize(self, x, scale, zp):
        """QUANTIZE (requantize) to new 8-bit params"""
        y = self._like(x, scale=scale, zp=zp)
        self.mb.op("QUANTIZE", [x], [y], OPT["QuantizeOptions"], Table())
        return y

    def concat(self, xs, axis=3):
        """CONCATENATION; int8 inputs are requantized to the first input's
        params first (what the converter does), uint8 ones are rescaled by the
        op itself (ConcatenationWithScaling)"""
        shp0, s0, z0 = self.meta[xs[0]]
        ins = []
        for x in xs:
            _, s, z = self.meta[x]
            if self.dtype == np.int8 and (s != s0 or z != z0):
                x = self.quantize(x, s0, z0)
            ins.append(x)
        shape = list(shp0)
        shape[axis] = sum(self.meta[x][0][axis] for x in ins)
        s_out = s0 if self.dtype == np.int8 else float(max(self.meta[x][1] for x in ins))
        z_out = z0 if self.dtype == np.int8 else self._act_zp()
        y = self.act_tensor(shape, s_out, z_out)
        self.mb.op("CONCATENATION", ins, [y], OPT["ConcatenationOptions"], Table().set(0, "i", axis).set(1, "b", 0))
        return y

    def pad(self, x, pads):
        """PAD with [[before, after]] per dim (quantized pad = output zero point)"""
        shp, _, _ = self.meta[x]
        pt = self.mb.tensor(self._name("paddings"), [len(shp), 2], np.int32, data=np.array(pads, np.int32))
        y = self._like(x, shape=[shp[d] + pads[d][0] + pads[d][1] for d in range(len(shp))])
        self.mb.op("PAD", [x, pt], [y], OPT["PadOptions"], Table())
        return y

    def relu(self, x, kind="RELU"):
        shp, s, z = self.meta[x]
        lo = {"RELU": 0.0, "RELU6": 0.0, "RELU_N1_TO_1": -1.0}[kind]
        hi = {"RELU": None, "RELU6": 6.0, "RELU_N1_TO_1": 1.0}[kind]
        qmin = -128 if self.dtype == np.int8 else 0
        span = (hi if hi is not None else s * 200.0) - lo
        scale = float(span / 255.0)
        y = self.act_tensor(shp, scale, int(qmin - round(lo / scale)))
        self.mb.op(kind, [x], [y])
        return y

    def logistic(self, x):
        zp = -128 if self.dtype == np.int8 else 0
        y = self._like(x, scale=1.0 / 256.0, zp=zp)
        self.mb.op("LOGISTIC", [x], [y])
        return y

    def softmax(self, x, beta=1.0):
        zp = -128 if self.dtype == np.int8 else 0
        y = self._like(x, scale=1.0 / 256.0, zp=zp)
        self.mb.op("SOFTMAX", [x], [y], OPT["SoftmaxOptions"], Table().set(0, "f", float(beta)))
        return y

    def resize(self, x, size, bilinear=False, align_corners=False, half_pixel_centers=False):
        shp, _, _ = self.meta[x]
        st = self.mb.tensor(self._name("size"), [2], np.int32, data=np.array(size, np.int32))
        y = self._like(x, shape=[shp[0], size[0], size[1], shp[3]])
        if bilinear:
            opt = Table().set(2, "b", int(align_corners)).set(3, "b", int(half_pixel_centers))
            self.mb.op("RESIZE_BILINEAR", [x, st], [y], OPT["ResizeBilinearOptions"], opt)
        else:
            opt = Table().set(0, "b", int(align_corners)).set(1, "b", int(half_pixel_centers))
            self.mb.op("RESIZE_NEAREST_NEIGHBOR", [x, st], [y], OPT["ResizeNearestNeighborOptions"], opt)
        return y

    def transpose_conv(self, x, out_c, k=3, stride=2, padding="SAME", bias=True):
        """TRANSPOSE_CONV (int8 per-channel): output = input * stride (SAME)
        or (input - 1) * stride + k (VALID)"""
        shp, s_in, _ = self.meta[x]
        b, h, w, c = shp
        oh = h * stride if padding == "SAME" else (h - 1) * stride + k
        ow = w * stride if padding == "SAME" else (w - 1) * stride + k
        s_out, zp = float(s_in) * 1.5, self._act_zp()
        K = max(1, k * k * c // (stride * stride))
        wt, ws = self._weights([out_c, k, k, c], out_c, 0, s_in, s_out, K)
        shape_t = self.mb.tensor(self._name("out_shape"), [4], np.int32, data=np.array([b, oh, ow, out_c], np.int32))
        ins = [shape_t, wt, x]
        if bias:
            ins.append(self._bias(out_c, s_in, ws, K))
        y = self.act_tensor([b, oh, ow, out_c], s_out, zp)
        opt = Table().set(0, "b", 0 if padding == "SAME" else 1).set(1, "i", stride).set(2, "i", stride)
        self.mb.op("TRANSPOSE_CONV", ins, [y], OPT["TransposeConvOptions"], opt)
        return y

    def dequantize(self, x):
        shp, _, _ = self.meta[x]
        y = self.mb.tensor(self._name("float"), shp, np.float32)
        self.mb.op("DEQUANTIZE", [x], [y], OPT["DequantizeOptions"], Table())
        self.fshape[y] = list(shp)
        return y

    def float_add(self, a, b, act="NONE"):
        """float32 ADD (a CPU-worker op: the GPU set is 8-bit only)"""
        y = self.mb.tensor(self._name("float"), self.fshape[a], np.float32)
        self.mb.op("ADD", [a, b], [y], OPT["AddOptions"], act_options(act))
        self.fshape[y] = list(self.fshape[a])
        return y

    def detection_postprocess(self, boxes_f, scores_f, anchors, num_classes, max_detections=25,
                              score_threshold=0.4, iou_threshold=0.5, scales=(10.0, 10.0, 5.0, 5.0)):
        """TFLite_Detection_PostProcess (CUSTOM; fast NMS, one class per
        detection): float box encodings [1,N,4], float class scores
        [1,N,C(+1)], constant anchors [N,4] (y, x, h, w) -> boxes, classes,
        scores, num_detections"""
        n = anchors.shape[0]
        a = self.mb.tensor(self._name("anchors"), [n, 4], np.float32, data=anchors.astype(np.float32))
        outs = [self.mb.tensor(self._name("detection_boxes"), [1, max_detections, 4], np.float32),
                self.mb.tensor(self._name("detection_classes"), [1, max_detections], np.float32),
                self.mb.tensor(self._name("detection_scores"), [1, max_detections], np.float32),
                self.mb.tensor(self._name("num_detections"), [1], np.float32)]
        opts = flexbuffer_map(dict(max_detections=int(max_detections), max_classes_per_detection=1,
                                   detections_per_class=100, use_regular_nms=False,
                                   nms_score_threshold=float(score_threshold), nms_iou_threshold=float(iou_threshold),
                                   num_classes=int(num_classes), y_scale=float(scales[0]), x_scale=float(scales[1]),
                                   h_scale=float(scales[2]), w_scale=float(scales[3])))
        self.mb.op("CUSTOM", [boxes_f, scores_f, a], outs, custom="TFLite_Detection_PostProcess",
                   custom_options=opts)
        for t, shp in zip(outs, ([1, max_detections, 4], [1, max_detections], [1, max_detections], [1])):
            self.fshape[t] = shp
        return outs

    def quantize_float(self, xf, scale, zp=None):
        """QUANTIZE float32 -> 8-bit"""
        y = self.act_tensor(self.fshape[xf], scale, self._act_zp() if zp is None else zp)
        self.mb.op("QUANTIZE", [xf], [y], OPT["QuantizeOptions"], Table())
        return y

    def build(self):
        return self.mb.build()


class FGraph:
    """Float graph builder with QGraph's method names: a TFLite fp16 model
    (post-training float16 quantization) - float32 activations, every
    constant stored as float16 behind a DEQUANTIZE op, float32 compute.
    Weights are He-initialised so activations stay O(1) through ReLU6."""

    def __init__(self, seed=0, name="model"):
        self.dtype = np.dtype(np.float16)
        self.rng = np.random.default_rng(seed)
        self.mb = ModelBuilder(name)
        self.n = 0
        self.meta = {}  # tensor -> (shape, None, None)

    def _name(self, kind):
        self.n += 1
        return "%s_%d" % (kind, self.n)

    def _act(self, shape, kind="act"):
        t = self.mb.tensor(self._name(kind), list(shape), np.float32)
        self.meta[t] = (list(shape), None, None)
        return t

    def _const(self, values, kind):
        """float16 constant + DEQUANTIZE -> float32 tensor"""
        v = np.asarray(values, np.float32)
        c = self.mb.tensor(self._name(kind + "_fp16"), list(v.shape), np.float16, data=v.astype(np.float16))
        y = self.mb.tensor(self._name(kind), list(v.shape), np.float32)
        self.mb.op("DEQUANTIZE", [c], [y], OPT["DequantizeOptions"], Table())
        return y

    def input(self, shape, scale=None, zp=None):
        t = self._act(shape, "input")
        self.mb.inputs.append(t)
        return t

    def output(self, t):
        self.mb.outputs.append(t)

    def conv(self, x, out_c, k=1, stride=1, act="RELU6", padding="SAME", dilation=1, out_scale=None,
             bias_offset_lsb=0):
        b, h, w, c = self.meta[x][0]
        K = k * k * c
        wt = self._const(self.rng.normal(0, np.sqrt(2.0 / K), (out_c, k, k, c)), "weights")
        bt = self._const(self.rng.normal(0, 0.05, out_c) + (bias_offset_lsb * 0.05 if bias_offset_lsb else 0), "bias")
        eff = (k - 1) * dilation + 1
        oh = (h + stride - 1) // stride if padding == "SAME" else (h + stride - eff) // stride
        ow = (w + stride - 1) // stride if padding == "SAME" else (w + stride - eff) // stride
        y = self._act([b, oh, ow, out_c])
        self.mb.op("CONV_2D", [x, wt, bt], [y], OPT["Conv2DOptions"], conv_options(padding, stride, act, dilation))
        return y

    def dwconv(self, x, k=3, stride=1, act="RELU6", padding="SAME", dm=1, dilation=1):
        b, h, w, c = self.meta[x][0]
        out_c = c * dm
        wt = self._const(self.rng.normal(0, np.sqrt(2.0 / (k * k)), (1, k, k, out_c)), "dw_weights")
        bt = self._const(self.rng.normal(0, 0.05, out_c), "dw_bias")
        eff = (k - 1) * dilation + 1
        oh = (h + stride - 1) // stride if padding == "SAME" else (h + stride - eff) // stride
        ow = (w + stride - 1) // stride if padding == "SAME" else (w + stride - eff) // stride
        y = self._act([b, oh, ow, out_c])
        self.mb.op("DEPTHWISE_CONV_2D", [x, wt, bt], [y], OPT["DepthwiseConv2DOptions"],
                   dw_options(padding, stride, act, dm, dilation))
        return y

    def add(self, a, b, act="NONE"):
        y = self._act(self.meta[a][0])
        self.mb.op("ADD", [a, b], [y], OPT["AddOptions"], act_options(act))
        return y

    def mul(self, a, b, act="NONE"):
        y = self._act(self.meta[a][0])
        self.mb.op("MUL", [a, b], [y], OPT["MulOptions"], act_options(act))
        return y

    def _pool(self, kind, x, filt, stride, padding):
        b, h, w, c = self.meta[x][0]
        oh = (h + stride - filt[0]) // stride if padding == "VALID" else (h + stride - 1) // stride
        ow = (w + stride - filt[1]) // stride if padding == "VALID" else (w + stride - 1) // stride
        y = self._act([b, oh, ow, c])
        self.mb.op(kind, [x], [y], OPT["Pool2DOptions"], pool_options(padding, stride, filt))
        return y

    def avgpool(self, x, filt, stride=1, padding="VALID"):
        return self._pool("AVERAGE_POOL_2D", x, filt, stride, padding)

    def maxpool(self, x, filt, stride, padding="SAME"):
        return self._pool("MAX_POOL_2D", x, filt, stride, padding)

    def reshape(self, x, shape):
        st = self.mb.tensor(self._name("shape"), [len(shape)], np.int32, data=np.array(shape, np.int32))
        y = self._act(list(shape))
        self.mb.op("RESHAPE", [x, st], [y], OPT["ReshapeOptions"], Table().set(0, "o", Vec("i", list(shape))))
        return y

    def fully_connected(self, x, units, act="NONE"):
        shp = self.meta[x][0]
        depth = shp[-1]
        rows = int(np.prod(shp)) // depth
        wt = self._const(self.rng.normal(0, np.sqrt(1.0 / depth), (units, depth)), "fc_weights")
        bt = self._const(self.rng.normal(0, 0.05, units), "fc_bias")
        y = self._act([rows, units])
        self.mb.op("FULLY_CONNECTED", [x, wt, bt], [y], OPT["FullyConnectedOptions"], act_options(act))
        return y

    def concat(self, xs, axis=3):
        shp = list(self.meta[xs[0]][0])
        shp[axis] = sum(self.meta[t][0][axis] for t in xs)
        y = self._act(shp)
        self.mb.op("CONCATENATION", list(xs), [y], OPT["ConcatenationOptions"], Table().set(0, "i", axis))
        return y

    def logistic(self, x):
        y = self._act(self.meta[x][0])
        self.mb.op("LOGISTIC", [x], [y])
        return y

    def softmax(self, x, beta=1.0):
        y = self._act(self.meta[x][0])
        self.mb.op("SOFTMAX", [x], [y], OPT["SoftmaxOptions"], Table().set(0, "f", float(beta)))
        return y

    def relu(self, x, kind="RELU"):
        y = self._act(self.meta[x][0])
        self.mb.op(kind, [x], [y])
        return y

    def build(self):
        return self.mb.build()


def _graph(dtype, seed, name):
    """QGraph for 8-bit models, FGraph for fp16-weight float models"""
    if np.dtype(dtype) == np.float16:
        return FGraph(seed, name)
    return QGraph(dtype, seed, name)


# ---------------------------------------------------------------------------
# BASELINE models
# ---------------------------------------------------------------------------
MNV2_BLOCKS = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1),
               (6, 160, 3, 2), (6, 320, 1, 1)]


def mobilenet_v2(dtype=np.int8, seed=0, size=224, batch=1, classes=1001, width=1.0):
    """MobileNetV2-1.0 with the topology of mobilenet_v2_1.0_224_quant.tflite
    (65 ops: 36 CONV_2D, 17 DEPTHWISE_CONV_2D, 10 ADD, AVERAGE_POOL_2D, RESHAPE)."""
    g = _graph(dtype, seed, "mobilenet_v2_%s" % np.dtype(dtype).name)
    ch = lambda c: max(8, int(c * width + 4) // 8 * 8)
    x = g.input([batch, size, size, 3])
    x = g.conv(x, ch(32), k=3, stride=2)
    c_in = ch(32)
    for t, c, n, s in MNV2_BLOCKS:
        for i in range(n):
            inp = x
            stride = s if i == 0 else 1
            h = x
            if t != 1:
                h = g.conv(h, c_in * t, k=1)
            h = g.dwconv(h, k=3, stride=stride)
            h = g.conv(h, ch(c), k=1, act="NONE")
            if stride == 1 and c_in == ch(c):
                h = g.add(h, inp)
            x = h
            c_in = ch(c)
    x = g.conv(x, 1280 if width <= 1.0 else ch(1280), k=1)
    k = size // 32
    x = g.avgpool(x, (k, k))
    x = g.conv(x, classes, k=1, act="NONE")
    x = g.reshape(x, [batch, classes])
    g.output(x)
    return g.build()


def mobilenet_v1(dtype=np.int8, seed=0, size=224, batch=1, classes=1001):
    """MobileNetV1-1.0 (config C1): conv + 13 depthwise-separable blocks."""
    g = _graph(dtype, seed, "mobilenet_v1_%s" % np.dtype(dtype).name)
    x = g.input([batch, size, size, 3])
    x = g.conv(x, 32, k=3, stride=2)
    for c, s in [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2), (512, 1), (512, 1),
                 (512, 1), (512, 1), (512, 1), (1024, 2), (1024, 1)]:
        x = g.dwconv(x, stride=s)
        x = g.conv(x, c, k=1)
    k = size // 32
    x = g.avgpool(x, (k, k))
    x = g.conv(x, classes, k=1, act="NONE")
    x = g.reshape(x, [batch, classes])
    g.output(x)
    return g.build()


# ---------------------------------------------------------------------------
# BASELINE C3 mix: detection / segmentation / pose heads on MobileNet trunks
# (synthetic weights, 224x224 inputs - "synthetic 224x224 batches", §8(d))
# ---------------------------------------------------------------------------
def _mnv2_trunk(g, x, out_stride=32, tap_expansion_at=None):
    """MobileNetV2 feature extractor.  out_stride 16 turns the last stride-2
    stage into stride 1 with dilation 2 (DeepLab).  Returns (features, taps):
    taps["expansion"] = the 1x1 expansion output of block `tap_expansion_at`
    (SSD's 'layer_15/expansion_output')."""
    x = g.conv(x, 32, k=3, stride=2)
    c_in, os_now, dil, taps, blk = 32, 2, 1, {}, 0
    for t, c, n, s in MNV2_BLOCKS:
        for i in range(n):
            inp, stride = x, (s if i == 0 else 1)
            if stride == 2 and os_now >= out_stride:
                stride, dil = 1, dil * 2
            elif stride == 2:
                os_now *= 2
            h = x
            if t != 1:
                h = g.conv(h, c_in * t, k=1)
                if blk == tap_expansion_at:
                    taps["expansion"] = h
            h = g.dwconv(h, k=3, stride=stride, dilation=dil)
            h = g.conv(h, c, k=1, act="NONE")
            if stride == 1 and c_in == c:
                h = g.add(h, inp)
            x, c_in, blk = h, c, blk + 1
    return x, taps


def ssd_mobilenet_v2(dtype=np.int8, seed=1, size=224, batch=1, classes=91):
    """SSD-MobileNetV2 (TF object-detection API layout): feature maps at
    layer_15/expansion_output (14x14x576) and the 1280-channel head (7x7),
    four extra 1x1 -> 3x3 s2 feature layers, 1x1 box / class predictors,
    RESHAPE + CONCATENATION of all anchors, LOGISTIC class scores.  The
    TFLite_Detection_PostProcess custom op (CPU NMS) is left out: outputs are
    box encodings [1,N,4] and class scores [1,N,classes]."""
    g = _graph(dtype, seed, "ssd_mobilenet_v2_%s" % np.dtype(dtype).name)
    x = g.input([batch, size, size, 3])
    feat, taps = _mnv2_trunk(g, x, tap_expansion_at=13)
    maps = [taps["expansion"], g.conv(feat, 1280, k=1)]
    y = maps[-1]
    for c1, c3 in ((256, 512), (128, 256), (128, 256), (64, 128)):
        y = g.conv(g.conv(y, c1, k=1), c3, k=3, stride=2)
        maps.append(y)
    boxes, scores = [], []
    for i, m in enumerate(maps):
        b, h, w, _ = g.meta[m][0]
        anchors = 3 if i == 0 else 6
        bx = g.conv(m, anchors * 4, k=1, act="NONE")
        cl = g.conv(m, anchors * classes, k=1, act="NONE")
        boxes.append(g.reshape(bx, [batch, h * w * anchors, 4]))
        scores.append(g.reshape(cl, [batch, h * w * anchors, classes]))
    g.output(g.concat(boxes, axis=1))
    g.output(g.logistic(g.concat(scores, axis=1)))
    return g.build()


def _round_filters(c, width):
    """EfficientNet channel rounding to a multiple of 8"""
    new = max(8, int(c * width + 4) // 8 * 8)
    if new < 0.9 * c * width:
        new += 8
    return new


# EfficientNet-B0 stages: (expand, kernel, stride, channels, repeats)
EFFNET_STAGES = [(1, 3, 1, 16, 1), (6, 3, 2, 24, 2), (6, 5, 2, 40, 2), (6, 3, 2, 80, 3), (6, 5, 1, 112, 3),
                 (6, 5, 2, 192, 4), (6, 3, 1, 320, 1)]


def efficientdet_anchors(size, levels=(3, 4, 5, 6, 7), anchor_scale=4.0):
    """normalised (ycenter, xcenter, h, w) per feature-map cell x 9 anchors,
    in the order the heads' RESHAPE lays them out"""
    out = []
    for lvl in levels:
        stride = 2 ** lvl
        n = -(-size // stride)
        for y in range(n):
            for x in range(n):
                for sc in (1.0, 2 ** (1 / 3), 2 ** (2 / 3)):
                    for rh, rw in ((1.0, 1.0), (1.4, 0.7), (0.7, 1.4)):
                        base = anchor_scale * stride * sc
                        out.append(((y + 0.5) * stride / size, (x + 0.5) * stride / size,
                                    base * rh / size, base * rw / size))
    return np.array(out, np.float32)


def efficientdet_lite2(dtype=np.int8, seed=4, size=448, batch=1, classes=90, fpn_channels=112, fpn_repeats=5,
                       head_repeats=3, max_detections=25, postprocess=True):
    """EfficientDet-Lite2 (BASELINE C4): EfficientNet-Lite2 backbone (width
    1.1, depth 1.2, ReLU6, no squeeze-excite), BiFPN P3-P7 with 112
    channels x 5 cells (sum fusion, separable convs, nearest upsampling,
    3x3/s2 max-pool downsampling), separable-conv class / box heads with 9
    anchors per cell, LOGISTIC scores, and TFLite_Detection_PostProcess
    (CUSTOM) on DEQUANTIZEd boxes / scores - the op the GPU worker cannot
    run, so the model analyzer splits the model there."""
    g = QGraph(dtype, seed, "efficientdet_lite2_%s" % np.dtype(dtype).name)
    x = g.input([batch, size, size, 3])
    y = g.conv(x, 32, k=3, stride=2)
    taps = []
    n_stages = len(EFFNET_STAGES)
    for si, (t, k, s_, c, r) in enumerate(EFFNET_STAGES):
        c = _round_filters(c, 1.1)
        reps = r if si in (0, n_stages - 1) else int(np.ceil(r * 1.2))
        for i in range(reps):
            stride = s_ if i == 0 else 1
            cin = g.meta[y][0][3]
            h = g.conv(y, cin * t, k=1) if t != 1 else y
            h = g.dwconv(h, k=k, stride=stride)
            h = g.conv(h, c, k=1, act="NONE")
            y = g.add(h, y) if stride == 1 and cin == c else h
        if si in (2, 4, 6):  # strides 8, 16, 32
            taps.append(y)
    F = fpn_channels
    p3, p4, p5 = (g.conv(t_, F, k=1, act="NONE") for t_ in taps)
    p6 = g.maxpool(g.conv(taps[2], F, k=1, act="NONE"), (3, 3), 2)
    p7 = g.maxpool(p6, (3, 3), 2)
    feats = [p3, p4, p5, p6, p7]

    def size_of(t):
        return tuple(g.meta[t][0][1:3])

    def sep(t, act="NONE"):
        return g.conv(g.dwconv(t, k=3, act="NONE"), F, k=1, act=act)

    def fuse(*ts):
        acc = ts[0]
        for i, t in enumerate(ts[1:]):
            acc = g.add(acc, t, act="RELU6" if i == len(ts) - 2 else "NONE")
        return sep(acc)

    for _ in range(fpn_repeats):
        td = [None] * 5
        td[4] = feats[4]
        for l in (3, 2, 1):
            td[l] = fuse(feats[l], g.resize(td[l + 1], size_of(feats[l])))
        out = [None] * 5
        out[0] = fuse(feats[0], g.resize(td[1], size_of(feats[0])))
        for l in (1, 2, 3):
            out[l] = fuse(feats[l], td[l], g.maxpool(out[l - 1], (3, 3), 2))
        out[4] = fuse(feats[4], g.maxpool(out[3], (3, 3), 2))
        feats = out

    boxes, scores = [], []
    for f in feats:
        b_, h, w, _ = g.meta[f][0]
        cl, bx = f, f
        for _ in range(head_repeats):
            cl = sep(cl, act="RELU6")
            bx = sep(bx, act="RELU6")
        # class prior: logits around -5.4, scale 4.6 / 60 (a few hundred anchors pass 0.4)
        cl = g.conv(g.dwconv(cl, k=3, act="NONE"), 9 * classes, k=1, act="NONE", out_scale=4.6 / 60,
                    bias_offset_lsb=-70)
        bx = g.conv(g.dwconv(bx, k=3, act="NONE"), 9 * 4, k=1, act="NONE")
        scores.append(g.reshape(cl, [batch, h * w * 9, classes]))
        boxes.append(g.reshape(bx, [batch, h * w * 9, 4]))
    box_enc = g.concat(boxes, axis=1)
    cls = g.logistic(g.concat(scores, axis=1))
    if not postprocess:
        g.output(box_enc)
        g.output(cls)
        return g.build()
    anchors = efficientdet_anchors(size)
    outs = g.detection_postprocess(g.dequantize(box_enc), g.dequantize(cls), anchors, classes,
                                   max_detections=max_detections)
    for o in outs:
        g.output(o)
    return g.build()


def deeplab_v3_mobilenet_v2(dtype=np.int8, seed=2, size=224, batch=1, classes=21):
    """DeepLabV3 with a MobileNetV2 trunk at output stride 16 (dilated last
    stages) and the mobile ASPP: image pooling (global AVERAGE_POOL_2D, 1x1
    conv, RESIZE_BILINEAR back) + a 1x1 branch, CONCATENATION, 1x1
    projection, 1x1 logits, RESIZE_BILINEAR x16 to the input size."""
    g = QGraph(dtype, seed, "deeplab_v3_mnv2_%s" % np.dtype(dtype).name)
    x = g.input([batch, size, size, 3])
    feat, _ = _mnv2_trunk(g, x, out_stride=16)
    fh = g.meta[feat][0][1]
    pool = g.conv(g.avgpool(feat, (fh, fh)), 256, k=1, act="RELU")
    pool = g.resize(pool, (fh, fh), bilinear=True, align_corners=True)
    aspp0 = g.conv(feat, 256, k=1, act="RELU")
    y = g.conv(g.concat([pool, aspp0], axis=3), 256, k=1, act="RELU")
    y = g.conv(y, classes, k=1, act="NONE")
    g.output(g.resize(y, (size, size), bilinear=True, align_corners=True))
    return g.build()


def posenet_mobilenet_v1(dtype=np.int8, seed=3, size=224, batch=1, keypoints=17):
    """PoseNet (multi-person, MobileNetV1 trunk at output stride 16): heatmap
    (LOGISTIC), offset and forward / backward displacement 1x1 heads."""
    g = QGraph(dtype, seed, "posenet_mnv1_%s" % np.dtype(dtype).name)
    x = g.input([batch, size, size, 3])
    x = g.conv(x, 32, k=3, stride=2)
    os_now, dil = 2, 1
    for c, s in [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2), (512, 1), (512, 1),
                 (512, 1), (512, 1), (512, 1), (1024, 2), (1024, 1)]:
        if s == 2 and os_now >= 16:
            s, dil = 1, dil * 2
        elif s == 2:
            os_now *= 2
        x = g.dwconv(x, stride=s, dilation=dil)
        x = g.conv(x, c, k=1)
    g.output(g.logistic(g.conv(x, keypoints, k=1, act="NONE")))
    g.output(g.conv(x, 2 * keypoints, k=1, act="NONE"))
    g.output(g.conv(x, 2 * (keypoints - 1), k=1, act="NONE"))
    g.output(g.conv(x, 2 * (keypoints - 1), k=1, act="NONE"))
    return g.build()


MIX_C3 = ("mobilenet_v2", "ssd_mobilenet_v2", "deeplab_v3_mobilenet_v2", "posenet_mobilenet_v1")


def int8_from_uint8(model_bytes):
    """Convert a uint8 per-tensor TFLite model to int8 per-channel with the
    same float semantics (what TFLite's converter emits for int8): activations
    shift by -128 (same scale), conv/dw filters re-quantised symmetric per
    output channel, biases re-scaled to in_scale*w_scale[c]."""
    from .tflite_reader_py import read  # local, dependency-free reader
    m = read(model_bytes)
    mb = ModelBuilder("int8 conversion of %s" % m["description"])
    tmap = {}
    new_w = {}
    # per-op filter / bias conversion
    for op in m["ops"]:
        if op["builtin"] in (OPC["CONV_2D"], OPC["DEPTHWISE_CONV_2D"]):
            x, w, b = op["inputs"][:3]
            tw, tb, tx = m["tensors"][w], m["tensors"][b], m["tensors"][x]
            wf = (tw["data"].astype(np.float32) - tw["zero_point"][0]) * tw["scale"][0]
            qdim = 0 if op["builtin"] == OPC["CONV_2D"] else 3
            axes = tuple(i for i in range(4) if i != qdim)
            amax = np.max(np.abs(wf), axis=axes)
            sc = np.where(amax > 0, amax / 127.0, 1.0).astype(np.float32)
            shp = [1, 1, 1, 1]
            shp[qdim] = -1
            wq = np.clip(np.round(wf / sc.reshape(shp)), -127, 127).astype(np.int8)
            bf = tb["data"].astype(np.float64) * tb["scale"][0]
            bsc = (np.float32(tx["scale"][0]) * sc).astype(np.float32)
            bq = np.round(bf / bsc.astype(np.float64)).astype(np.int32)
            new_w[w] = (wq, sc, qdim)
            new_w[b] = (bq, bsc, 0)
    for i, t in enumerate(m["tensors"]):
        if i in new_w:
            data, sc, qd = new_w[i]
            tmap[i] = mb.tensor(t["name"], t["shape"], data.dtype, scale=sc, zero_point=[0] * len(sc),
                                qdim=qd, data=data)
        elif t["type"] == T_UINT8:
            zp = [z - 128 for z in t["zero_point"]] if t["zero_point"] is not None else None
            data = None if t["data"] is None else (t["data"].astype(np.int16) - 128).astype(np.int8)
            tmap[i] = mb.tensor(t["name"], t["shape"], np.int8, scale=t["scale"], zero_point=zp, data=data)
        else:
            dt = {T_INT32: np.int32, T_FLOAT32: np.float32, T_INT8: np.int8}[t["type"]]
            tmap[i] = mb.tensor(t["name"], t["shape"], dt, scale=t["scale"], zero_point=t["zero_point"],
                                data=t["data"])
    for op in m["ops"]:
        mb.op(op["builtin"], [tmap[i] if i >= 0 else -1 for i in op["inputs"]], [tmap[i] for i in op["outputs"]],
              op["options_type"], op["options"])
    mb.inputs = [tmap[i] for i in m["inputs"]]
    mb.outputs = [tmap[i] for i in m["outputs"]]
    return mb.build()
