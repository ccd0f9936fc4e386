"""Wire-format decoders: Kubernetes objects as the apiserver serves them (JSON) into the
boundary structs, through the C ABI (ke_decode_* in libkoordeval.so; no Python re-implementation runs here).

    node = decode_node(node_json)                  -> abi.Node
    nm, pms, n_pm, aggs, n_agg = decode_node_metric(nodemetric_json)   (the Evaluator.set_nodemetric layout)
    pod = decode_pod(pod_json, xres_names)         -> abi.Pod
    devices, (has_table, honor, partitions) = decode_device(device_json)
    zones, cpus = decode_nrt(nrt_json, node)       (patches the NRT-side fields of `node`)
    hints = decode_pod_device_hints(pod_json)       -> abi.PodDeviceHints or None (no hint annotations)
    well_planned, model_key = decode_device_flags(device_json, node_json)
    rsv, alloc, resources, node_name = decode_reservation(reservation_json, xres_names)
Objects may be given as dicts (serialised with json.dumps) or JSON text.
"""
import ctypes as C
import json

import numpy as np

from . import abi


class DecodeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"koord-eval decode error {code}: {msg}")
        self.code = code


def _lib():
    return abi.load_library()


def _text(obj):
    s = obj if isinstance(obj, (str, bytes)) else json.dumps(obj)
    return s.encode() if isinstance(s, str) else s


def _check(lib, rc):
    if rc != abi.OK:
        raise DecodeError(rc, lib.ke_last_error().decode())


def parse_quantity(s):
    """(Value(), MilliValue()) of a resource.Quantity string."""
    lib = _lib()
    v, m = abi.i64(), abi.i64()
    _check(lib, lib.ke_quantity_parse(s.encode(), C.byref(v), C.byref(m)))
    return v.value, m.value


def pod_key(namespace, name):
    return _lib().ke_pod_key(namespace.encode(), name.encode())


def decode_node(obj):
    lib = _lib()
    t = _text(obj)
    n = abi.Node()
    _check(lib, lib.ke_decode_node(t, len(t), C.byref(n)))
    return n


def decode_node_metric(obj, pm_cap=4096, agg_cap=16):
    lib = _lib()
    t = _text(obj)
    nm = abi.NodeMetric()
    pms = (abi.PodMetric * max(pm_cap, 1))()
    aggs = (abi.AggregatedUsage * max(agg_cap, 1))()
    n_pm, n_agg = abi.i32(), abi.i32()
    _check(lib, lib.ke_decode_node_metric(t, len(t), C.byref(nm), pm_cap, pms, C.byref(n_pm), agg_cap, aggs,
                                          C.byref(n_agg)))
    return nm, pms, n_pm.value, aggs, n_agg.value


def decode_pod(obj, xres_names=()):
    lib = _lib()
    t = _text(obj)
    names = (C.c_char_p * max(len(xres_names), 1))(*[n.encode() for n in xres_names])
    p = abi.Pod()
    _check(lib, lib.ke_decode_pod(t, len(t), len(xres_names), names, C.byref(p)))
    return p


def decode_reservation(obj, xres_names=()):
    """Reservation -> (abi.Reservation with node = -1, RESERVATION_ALLOC_DTYPE record of the reserve pod's holdings,
    RESERVATION_RESOURCE_DTYPE entries beyond cpu / memory, status.nodeName).  xres_names[id] = the resource name of
    id (None = no name)."""
    lib = _lib()
    t = _text(obj)
    names = (C.c_char_p * max(len(xres_names), 1))(*[n.encode() if n else None for n in xres_names])
    r = abi.Reservation()
    a = np.zeros(1, abi.RESERVATION_ALLOC_DTYPE)
    res = np.zeros(abi.MAX_XRES + 1, abi.RESERVATION_RESOURCE_DTYPE)
    n = abi.i32()
    node = C.create_string_buffer(256)
    _check(lib, lib.ke_decode_reservation(t, len(t), len(xres_names), names, C.byref(r), abi.ptr(a), len(res),
                                          abi.ptr(res), C.byref(n), node, 256))
    return r, a[0], res[:n.value].copy(), node.value.decode()


def decode_device(obj, cap=3 * abi.MAX_MINORS, part_cap=abi.MAX_GPU_PARTITIONS):
    lib = _lib()
    t = _text(obj)
    devs = np.zeros(cap, abi.DEVICE_DTYPE)
    parts = np.zeros(part_cap, abi.GPU_PARTITION_DTYPE)
    n, n_parts, has_table, honor = abi.i32(), abi.i32(), abi.i32(), abi.i32()
    _check(lib, lib.ke_decode_device(t, len(t), cap, abi.ptr(devs), C.byref(n), part_cap, abi.ptr(parts),
                                     C.byref(n_parts), C.byref(has_table), C.byref(honor)))
    return devs[:n.value], (bool(has_table.value), bool(honor.value), parts[:n_parts.value])


def decode_nrt(obj, node):
    """NodeResourceTopology -> (zones NUMA_ZONE_DTYPE, cpus CPU_DTYPE); patches the NRT-side fields of `node`."""
    lib = _lib()
    t = _text(obj)
    zones = np.zeros(abi.MAX_NUMA, abi.NUMA_ZONE_DTYPE)
    cpus = np.zeros(abi.MAX_CPUS, abi.CPU_DTYPE)
    nz, nc = abi.i32(), abi.i32()
    _check(lib, lib.ke_decode_nrt(t, len(t), C.byref(node), abi.MAX_NUMA, abi.ptr(zones), C.byref(nz), abi.MAX_CPUS,
                                  abi.ptr(cpus), C.byref(nc)))
    return zones[:nz.value], cpus[:nc.value]


def label_id(text):
    """ke_label_id: the process-wide id of a label key / value string (0 for an empty one)."""
    return _lib().ke_label_id(text.encode())


def decode_pod_device_hints(obj):
    lib = _lib()
    t = _text(obj)
    h = abi.PodDeviceHints()
    present = abi.i32()
    _check(lib, lib.ke_decode_pod_device_hints(t, len(t), C.byref(h), C.byref(present)))
    return h if present.value else None


def decode_device_flags(device_obj=None, node_obj=None):
    lib = _lib()
    dt = _text(device_obj) if device_obj is not None else None
    nt = _text(node_obj) if node_obj is not None else None
    w, k = abi.i32(), abi.i32()
    _check(lib, lib.ke_decode_device_flags(dt, len(dt) if dt else 0, nt, len(nt) if nt else 0, C.byref(w), C.byref(k)))
    return bool(w.value), k.value
