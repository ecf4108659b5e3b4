"""Host-path copy rate vs. the NUMA node of the host buffers (VERDICT r05
item 3).  Reports the GPU's NUMA node, the process's CPUs and their nodes,
where the pages of the frame and the map landed (/proc/self/numa_maps), and
times the plug-in's call (16384^2 RGB, N = 8: pageable frame -> dcte_energy_map
-> pageable map) with the buffers first touched from each node's CPUs in
turn, next to the bare copy rates of the same bytes (registered, one
direction at a time and both at once).

    python tools/host_numa.py
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def node_cpus():
    base = "/sys/devices/system/node"
    out = {}
    for d in sorted(os.listdir(base)) if os.path.isdir(base) else []:
        if d.startswith("node") and d[4:].isdigit():
            txt = open(os.path.join(base, d, "cpulist")).read().strip()
            cpus = set()
            for part in txt.split(","):
                if not part:
                    continue
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
            out[int(d[4:])] = cpus
    return out


def pages_by_node(addr, nbytes):
    """node -> pages of the VMA(s) overlapping [addr, addr + nbytes)"""
    vmas = []
    for line in open("/proc/self/maps"):
        a, b = (int(x, 16) for x in line.split()[0].split("-"))
        if b > addr and a < addr + nbytes:
            vmas.append(a)
    res = {}
    for line in open("/proc/self/numa_maps"):
        f = line.split()
        if int(f[0], 16) in vmas:
            for tok in f[2:]:
                if tok.startswith("N") and "=" in tok:
                    k, v = tok[1:].split("=")
                    res[int(k)] = res.get(int(k), 0) + int(v)
    return res


def main():
    import numpy as np
    import torch
    import dctenergy
    from dctenergy import synth
    S = 16384
    props = torch.cuda.get_device_properties(0)
    bdf = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
    try:
        gpu_node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
    except OSError:
        gpu_node = None
    nodes = node_cpus()
    allowed = os.sched_getaffinity(0)
    info = {"gpu_bdf": bdf, "gpu_numa_node": gpu_node, "nodes": len(nodes),
            "allowed_cpus_per_node": {k: len(v & allowed) for k, v in nodes.items()},
            "cpu_model": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                               if l.startswith("model name")), None)}
    print(json.dumps(info), flush=True)
    src = synth.natural_rows(0, S, S, 3, seed=0, device="cuda").cpu().numpy()
    torch.cuda.empty_cache()
    hip = ctypes.CDLL("libamdhip64.so.7")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    hip.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [vp]
    hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
    hip.hipStreamSynchronize.argtypes = [vp]
    s1, s2 = vp(), vp()
    hip.hipStreamCreate(ctypes.byref(s1))
    hip.hipStreamCreate(ctypes.byref(s2))
    d_px = torch.empty((S, S, 3), dtype=torch.uint8, device="cuda")
    d_out = torch.empty((S, S), dtype=torch.float32, device="cuda")

    def bare(px, out):
        hip.hipHostRegister(px.ctypes.data, px.nbytes, 0)
        hip.hipHostRegister(out.ctypes.data, out.nbytes, 0)
        r = {}
        for name, fn in (("h2d", lambda: hip.hipMemcpyAsync(d_px.data_ptr(), px.ctypes.data, px.nbytes, 1, s1)),
                         ("d2h", lambda: hip.hipMemcpyAsync(out.ctypes.data, d_out.data_ptr(), out.nbytes, 2, s2)),
                         ("both", lambda: (hip.hipMemcpyAsync(d_px.data_ptr(), px.ctypes.data, px.nbytes, 1, s1),
                                           hip.hipMemcpyAsync(out.ctypes.data, d_out.data_ptr(), out.nbytes, 2, s2)))):
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                fn()
                hip.hipStreamSynchronize(s1)
                hip.hipStreamSynchronize(s2)
                ts.append((time.perf_counter() - t0) * 1e3)
            r[name + "_ms"] = round(min(ts), 2)
        hip.hipHostUnregister(px.ctypes.data)
        hip.hipHostUnregister(out.ctypes.data)
        return r

    with dctenergy.Context(ngpus=1) as ctx:
        cases = [("as allocated", None)] + [(f"first touch on node {k}", v & allowed)
                                             for k, v in nodes.items() if v & allowed]
        for name, cpus in cases:
            keep = os.sched_getaffinity(0)
            if cpus:
                os.sched_setaffinity(0, cpus)
            px = np.empty_like(src)
            px[...] = src
            out = np.empty((S, S), np.float32)
            out[...] = 0
            if cpus:
                os.sched_setaffinity(0, keep)
            ctx.energy_map(px, 8, 0.3, 0.7, out=out)
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                ctx.energy_map(px, 8, 0.3, 0.7, out=out)
                ts.append((time.perf_counter() - t0) * 1e3)
            r = {"case": name, "call_ms": round(sorted(ts)[1], 2),
                 "px_pages_by_node": pages_by_node(px.ctypes.data, px.nbytes),
                 "out_pages_by_node": pages_by_node(out.ctypes.data, out.nbytes)}
            r.update(bare(px, out))
            print(json.dumps(r), flush=True)
            del px, out


if __name__ == "__main__":
    main()
