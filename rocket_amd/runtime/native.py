"""ctypes bindings of ``librocket_runtime.so`` (``native/runtime/*.cpp``): RCCL communicator +
bucket reducer (comm.cpp), the host batch assembler (loader.cpp) and the launch-list replay of
captured HIP graphs (launchlist.cpp)."""

from __future__ import annotations

import ctypes

from rocket_amd.ops import _lib

c_void_p, c_int, c_int64, c_char_p = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_char_p
P = ctypes.POINTER(ctypes.c_void_p)

RUNTIME_SIGS = {
    "rkr_last_error": (c_char_p, []),
    "rkr_unique_id_bytes": (c_int, []),
    "rkr_unique_id": (c_int, [c_void_p]),
    "rkr_comm_init": (c_int, [P, c_int, c_int, c_void_p, c_int]),
    "rkr_comm_destroy": (c_int, [c_void_p]),
    "rkr_comm_abort": (c_int, [c_void_p]),
    "rkr_all_reduce": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "rkr_broadcast": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "rkr_all_gather": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "rkr_reduce_scatter": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "rkr_reducer_create": (c_int, [P, c_void_p, c_int]),
    "rkr_reducer_set_bucket": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int]),
    "rkr_reducer_launch": (c_int, [c_void_p, c_int, c_void_p]),
    "rkr_reducer_join": (c_int, [c_void_p, c_void_p]),
    "rkr_reducer_destroy": (c_int, [c_void_p]),
    "rkl_create": (c_int, [P, c_int, c_void_p, c_void_p, c_int64, c_int, c_int]),
    "rkl_submit": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_void_p]),
    "rkl_wait": (c_int, [c_void_p, c_int]),
    "rkl_destroy": (c_int, [c_void_p]),
    "rkg_last_error": (c_char_p, []),
    "rkg_create": (c_int, [P, c_void_p]),
    "rkg_describe": (c_int64, [c_void_p, c_char_p, c_int64]),
    "rkg_size": (c_int, [c_void_p]),
    "rkg_kind": (c_int, [c_void_p, c_int]),
    "rkg_launch": (c_int, [c_void_p, c_void_p]),
    "rkg_destroy": (c_int, [c_void_p]),
}


class RuntimeError_(RuntimeError):
    pass


def runtime():
    return _lib._load("rocket_runtime", RUNTIME_SIGS)


def check(code: int, what: str) -> None:
    if code != 0:
        msg = runtime().rkr_last_error()
        raise RuntimeError_(f"{what} failed ({code}): {msg.decode() if msg else ''}")


class LaunchList:
    """Launch-list replay of a captured graph (``native/runtime/launchlist.cpp``): the graph's nodes
    re-issued as plain stream launches, avoiding hipGraphLaunch's fixed boundary cost.  Holds a
    reference to the ``torch.cuda.CUDAGraph`` (captured with ``keep_graph=True``) whose node
    argument arrays the list points into.  ``LaunchList.build`` returns ``(list, None)`` or
    ``(None, reason)`` when a node type is not supported (the caller keeps ``graph.replay()``)."""

    def __init__(self, graph, handle):
        self._graph = graph
        self._h = handle
        rt = runtime()
        self._launch = rt.rkg_launch
        self._destroy = rt.rkg_destroy
        self.size = rt.rkg_size(handle)
        self.kinds = [rt.rkg_kind(handle, i) for i in range(self.size)]

    @classmethod
    def build(cls, graph):
        rt = runtime()
        h = ctypes.c_void_p()
        code = rt.rkg_create(ctypes.byref(h), ctypes.c_void_p(graph.raw_cuda_graph()))
        if code != 0:
            msg = rt.rkg_last_error()
            return None, (msg.decode() if msg else f"rkg_create failed ({code})")
        return cls(graph, h.value), None

    def launch(self, stream: int) -> None:
        code = self._launch(self._h, stream)
        if code != 0:
            msg = runtime().rkg_last_error()
            raise RuntimeError_(f"launch-list replay failed ({code}): {msg.decode() if msg else ''}")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            try:
                self._destroy(h)
            except Exception:
                pass


def describe_graph(graph):
    """Structure of a captured graph (``torch.cuda.CUDAGraph`` with ``keep_graph=True``):
    ``(nodes, edges)`` with ``nodes[i] = (type, kernel name or "-")`` and ``edges = [(from, to)]``
    (``native/runtime/launchlist.cpp`` ``rkg_describe``)."""
    rt = runtime()
    g = ctypes.c_void_p(graph.raw_cuda_graph())
    need = rt.rkg_describe(g, None, 0)
    if need < 0:
        raise RuntimeError_("rkg_describe failed")
    buf = ctypes.create_string_buffer(int(need))
    rt.rkg_describe(g, buf, need)
    nodes, edges = [], []
    for line in buf.value.decode(errors="replace").splitlines():
        parts = line.split(" ", 3)
        if parts[0] == "N":
            nodes.append((int(parts[2]), parts[3] if len(parts) > 3 else "-"))
        elif parts[0] == "E":
            edges.append((int(parts[1]), int(parts[2])))
    return nodes, edges
