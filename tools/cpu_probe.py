#!/usr/bin/env python3
"""tools/cpu_probe.py -- what CPU the GPU box's host has, how many of its cores this job may use, and
how the reference harness (oracle/_ref/ref_harness bench_mt: the reference's shipped RNG, persistent
thread pool) scales with threads on it.  One JSON line per measurement into gpurun_out/cpu_probe.jsonl.
"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def read(p):
    try:
        return open(p).read().strip()
    except OSError:
        return None


def topology():
    cpus = sorted(os.sched_getaffinity(0))
    pk = {}
    for c in range(os.cpu_count() or 0):
        pkg = read(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id")
        core = read(f"/sys/devices/system/cpu/cpu{c}/topology/core_id")
        if pkg is None:
            continue
        pk.setdefault(pkg, set()).add(core)
    model = None
    for line in (read("/proc/cpuinfo") or "").splitlines():
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    return {"model": model, "logical_cpus": os.cpu_count(), "affinity": len(cpus),
            "sockets": len(pk), "physical_cores_per_socket": {k: len(v) for k, v in pk.items()},
            "cgroup_cpu_max": read("/sys/fs/cgroup/cpu.max"), "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def main():
    out = os.path.join(REPO, "gpurun_out", "cpu_probe.jsonl")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    f = open(out, "a")
    topo = topology()
    print(json.dumps(topo), flush=True)
    f.write(json.dumps(topo) + "\n")
    import _oracle as O
    tmp = tempfile.mkdtemp(prefix="rt_probe_")
    for (name, raw, _, _) in O.cornell_meshes():
        with open(os.path.join(tmp, name + ".obj"), "w") as g:
            for v in raw.reshape(-1, 3):
                g.write("v %r %r %r\n" % tuple(float(c) for c in v))
            for i in range(raw.shape[0]):
                g.write("f %d %d %d\n" % (3 * i + 1, 3 * i + 2, 3 * i + 3))
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    threads = [int(x) for x in (sys.argv[1:] or ["1", "8", "16", "32", "64"])]
    for t in threads:
        spp = max(1, t // 4)
        r = subprocess.run([harness, "bench_mt", tmp, "", "1920", "1080", str(spp), "0.8", str(t)], capture_output=True, text=True,
                           timeout=300)
        tok = r.stdout.split()
        rec = {"threads": t, "spp": spp, "samples": int(tok[2]), "seconds": float(tok[4]),
               "msamples_per_s": int(tok[2]) / float(tok[4]) / 1e6}
        rec["per_thread"] = rec["msamples_per_s"] / t
        print(json.dumps(rec), flush=True)
        f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
