"""List the nodes of a captured torch.cuda.CUDAGraph (kept with enable_debug_mode or keep_graph):
type, kernel symbol, grid / block, memset extent, and the indices of each node's dependencies.

    from graph_nodes import describe
    lines = describe(g.raw_cuda_graph())
"""
import ctypes

_hip = None


class Dim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint), ("y", ctypes.c_uint), ("z", ctypes.c_uint)]


class KernelNodeParams(ctypes.Structure):
    _fields_ = [("blockDim", Dim3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p), ("gridDim", Dim3),
                ("kernelParams", ctypes.c_void_p), ("sharedMemBytes", ctypes.c_uint)]


class MemsetParams(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("elementSize", ctypes.c_uint), ("height", ctypes.c_size_t),
                ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]


TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait", 7: "record"}


def hip():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipKernelNameRefByPtr.restype = ctypes.c_char_p
        _hip.hipKernelNameRefByPtr.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return _hip


def describe(graph):
    h = hip()
    g = ctypes.c_void_p(graph)
    n = ctypes.c_size_t(0)
    assert h.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert h.hipGraphGetNodes(g, nodes, ctypes.byref(n)) == 0
    index = {nodes[i]: i for i in range(n.value)}
    out = []
    for i in range(n.value):
        nd = ctypes.c_void_p(nodes[i])
        t = ctypes.c_int(-1)
        h.hipGraphNodeGetType(nd, ctypes.byref(t))
        nd_deps = ctypes.c_size_t(0)
        h.hipGraphNodeGetDependencies(nd, None, ctypes.byref(nd_deps))
        deps = (ctypes.c_void_p * max(1, nd_deps.value))()
        h.hipGraphNodeGetDependencies(nd, deps, ctypes.byref(nd_deps))
        dl = [index.get(deps[k], -1) for k in range(nd_deps.value)]
        desc = TYPES.get(t.value, str(t.value))
        if t.value == 0:
            p = KernelNodeParams()
            h.hipGraphKernelNodeGetParams(nd, ctypes.byref(p))
            name = h.hipKernelNameRefByPtr(ctypes.c_void_p(p.func), None)
            name = name.decode(errors="replace") if name else hex(p.func or 0)
            desc += f" {name[:110]} grid=({p.gridDim.x},{p.gridDim.y},{p.gridDim.z}) block={p.blockDim.x} " \
                    f"lds={p.sharedMemBytes}"
        elif t.value == 2:
            p = MemsetParams()
            h.hipGraphMemsetNodeGetParams(nd, ctypes.byref(p))
            desc += f" dst={hex(p.dst or 0)} width={p.width} elem={p.elementSize} h={p.height} value={p.value}"
        out.append(f"{i:4d} deps={dl} {desc}")
    return out
