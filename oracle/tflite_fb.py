"""Minimal, dependency-free reader for TFLite schema-v3 flatbuffers.

ORACLE / TEST INFRASTRUCTURE ONLY.  Nothing in the product (`band_amd/`) may
import this module; the product has its own C++ reader
(`band_amd/csrc/backend/hip/tflite_reader.cc`).  Two independent readers let
each check the other.

The reference loads models through `tflite::FlatBufferModel::BuildFromFile`
(`band/backend/tfl/model.cc:25-32`), i.e. the third-party TFLite 2.9.2 schema
(`tensorflow/lite/schema/schema.fbs`, not vendored in /root/reference).  The
field indices used below are the schema's table slots.
"""
import struct

import numpy as np

# schema TensorType -> numpy dtype
TENSOR_TYPE_NP = {
    0: np.float32, 1: np.float16, 2: np.int32, 3: np.uint8, 4: np.int64,
    6: np.bool_, 7: np.int16, 9: np.int8, 10: np.float64,
}
TENSOR_TYPE_NAME = {0: "float32", 1: "float16", 2: "int32", 3: "uint8",
                    4: "int64", 5: "string", 6: "bool", 7: "int16",
                    9: "int8", 10: "float64"}

# BuiltinOperator codes (schema.fbs enum BuiltinOperator)
OP = dict(ADD=0, AVERAGE_POOL_2D=1, CONCATENATION=2, CONV_2D=3,
          DEPTHWISE_CONV_2D=4, DEQUANTIZE=6, FULLY_CONNECTED=9, LOGISTIC=14,
          MAX_POOL_2D=17, MUL=18, RELU=19, RELU_N1_TO_1=20, RELU6=21, RESHAPE=22,
          RESIZE_BILINEAR=23, SOFTMAX=25, CUSTOM=32, PAD=34, MEAN=40, SUB=41,
          SQUEEZE=43, PADV2=60, TRANSPOSE_CONV=67, RESIZE_NEAREST_NEIGHBOR=97,
          QUANTIZE=114, HARD_SWISH=117)
OP_NAME = {v: k for k, v in OP.items()}


class Table:
    __slots__ = ("buf", "pos", "vt", "vt_len")

    def __init__(self, buf, pos):
        self.buf = buf
        self.pos = pos
        self.vt = pos - struct.unpack_from("<i", buf, pos)[0]
        self.vt_len = struct.unpack_from("<H", buf, self.vt)[0]

    def _off(self, slot):
        o = 4 + 2 * slot
        if o >= self.vt_len:
            return 0
        return struct.unpack_from("<H", self.buf, self.vt + o)[0]

    def has(self, slot):
        return self._off(slot) != 0

    def scalar(self, slot, fmt, default=0):
        o = self._off(slot)
        if not o:
            return default
        return struct.unpack_from("<" + fmt, self.buf, self.pos + o)[0]

    def _deref(self, slot):
        o = self._off(slot)
        if not o:
            return None
        p = self.pos + o
        return p + struct.unpack_from("<I", self.buf, p)[0]

    def table(self, slot):
        p = self._deref(slot)
        return None if p is None else Table(self.buf, p)

    def string(self, slot):
        p = self._deref(slot)
        if p is None:
            return None
        n = struct.unpack_from("<I", self.buf, p)[0]
        return bytes(self.buf[p + 4:p + 4 + n]).decode("utf-8", "replace")

    def vector(self, slot, fmt):
        p = self._deref(slot)
        if p is None:
            return None
        n = struct.unpack_from("<I", self.buf, p)[0]
        dt = np.dtype("<" + fmt)
        return np.frombuffer(self.buf, dtype=dt, count=n, offset=p + 4)

    def table_vector(self, slot):
        p = self._deref(slot)
        if p is None:
            return []
        n = struct.unpack_from("<I", self.buf, p)[0]
        out = []
        for i in range(n):
            e = p + 4 + 4 * i
            out.append(Table(self.buf, e + struct.unpack_from("<I", self.buf, e)[0]))
        return out


class Tensor:
    def __init__(self, t, buffers, idx):
        self.index = idx
        shape = t.vector(0, "i4")
        self.shape = [] if shape is None else [int(x) for x in shape]
        self.type = t.scalar(1, "b", 0)
        self.buffer = t.scalar(2, "I", 0)
        self.name = t.string(3) or ""
        q = t.table(4)
        self.scale = None
        self.zero_point = None
        self.quantized_dimension = 0
        if q is not None:
            s = q.vector(2, "f4")
            z = q.vector(3, "i8")
            if s is not None and len(s):
                self.scale = np.array(s, dtype=np.float32)
                self.zero_point = (np.array(z, dtype=np.int64) if z is not None
                                   else np.zeros(len(s), np.int64))
            self.quantized_dimension = q.scalar(6, "i", 0)
        self.data = None
        b = buffers[self.buffer] if self.buffer < len(buffers) else None
        if b is not None:
            d = b.vector(0, "u1")
            if d is not None and len(d):
                self.data = np.frombuffer(bytes(d), dtype=TENSOR_TYPE_NP[self.type]).reshape(self.shape)

    @property
    def is_const(self):
        return self.data is not None

    @property
    def np_dtype(self):
        return TENSOR_TYPE_NP[self.type]


class Operator:
    def __init__(self, o, opcodes):
        self.opcode_index = o.scalar(0, "I", 0)
        self.builtin, self.custom = opcodes[self.opcode_index]
        ins = o.vector(1, "i4")
        outs = o.vector(2, "i4")
        self.inputs = [] if ins is None else [int(x) for x in ins]
        self.outputs = [] if outs is None else [int(x) for x in outs]
        self.options_type = o.scalar(3, "B", 0)
        self.options = o.table(4)
        co = o.vector(5, "u1")
        self.custom_options = bytes(co) if co is not None else b""

    @property
    def name(self):
        return OP_NAME.get(self.builtin, "OP%d" % self.builtin)


class Model:
    """One .tflite file: primary subgraph's tensors and operators."""

    def __init__(self, data):
        self.buf = bytes(data)
        root = Table(self.buf, struct.unpack_from("<I", self.buf, 0)[0])
        self.version = root.scalar(0, "I", 0)
        self.opcodes = []
        for oc in root.table_vector(1):
            dep = oc.scalar(0, "b", 0)
            code = oc.scalar(3, "i", 0)
            self.opcodes.append((max(dep, code), oc.string(1)))
        buffers = root.table_vector(4)
        sg = root.table_vector(2)[0]
        self.tensors = [Tensor(t, buffers, i) for i, t in enumerate(sg.table_vector(0))]
        self.inputs = [int(x) for x in sg.vector(1, "i4")]
        self.outputs = [int(x) for x in sg.vector(2, "i4")]
        self.operators = [Operator(o, self.opcodes) for o in sg.table_vector(3)]

    @classmethod
    def from_path(cls, path):
        with open(path, "rb") as f:
            return cls(f.read())
