#!/usr/bin/env python3
"""How the reference's CPU renderer scales with threads on this host (the evidence behind bench.py's
one-socket estimate, which multiplies the per-thread rate at the job's CPU share by the physical cores
of one socket).

oracle/_ref/ref_harness bench_mt (the reference's MC/ code, shipped RNG, C4 Cornell frame) is timed
  * at 1, 2, 4, 8 and 16 threads, each thread pinned to its own physical core (one CPU per core);
  * at 2 threads on the two SMT siblings of one core, against 1 thread on that core -- what SMT adds
    to a core, which the linear one-thread-per-core estimate leaves out.
CPU only (no GPU call).  One JSON object on stdout.

    python tools/cpu_scaling.py [--seconds 4]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return None


def topology():
    """(package, core) -> sorted CPUs of the affinity mask"""
    cores = {}
    for c in sorted(os.sched_getaffinity(0)):
        key = (read(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"), read(f"/sys/devices/system/cpu/cpu{c}/topology/core_id"))
        cores.setdefault(key, []).append(c)
    return cores


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0, help="CPU work per measurement")
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    a = ap.parse_args()
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        sys.exit("oracle/_ref/ref_harness is not built (make -C oracle ref)")
    import _oracle as O
    cores = topology()
    pkg0 = sorted(k for k in cores if k[0] == sorted(cores)[0][0])
    one_per_core = [cores[k][0] for k in pkg0]   # one CPU of each physical core of the first package
    smt_core = next((cores[k] for k in pkg0 if len(cores[k]) >= 2), None)
    tmp = tempfile.mkdtemp(prefix="rt_cpu_")
    try:
        for (name, raw, _, _) in O.cornell_meshes():
            with open(os.path.join(tmp, name + ".obj"), "w") as f:
                for v in raw.reshape(-1, 3):
                    f.write("v %r %r %r\n" % tuple(float(c) for c in v))
                for i in range(raw.shape[0]):
                    f.write("f %d %d %d\n" % (3 * i + 1, 3 * i + 2, 3 * i + 3))

        def run(cpus, spp):
            r = subprocess.run([harness, "bench_mt", tmp, "", str(a.W), str(a.H), str(spp), "0.8", str(len(cpus))],
                               check=True, capture_output=True, text=True, preexec_fn=lambda: os.sched_setaffinity(0, cpus))
            tok = r.stdout.split()
            return int(tok[2]) / float(tok[4]) / 1e6   # Msamples/s (frames only)

        # spp for ~`seconds` at one thread
        r1 = run(one_per_core[:1], 1)
        spp1 = max(1, int(a.seconds * r1 * 1e6 / (a.W * a.H)))
        out = {"host_cpus_in_affinity": sum(len(v) for v in cores.values()), "physical_cores_first_package": len(pkg0),
               "cgroup_cpu_max": read("/sys/fs/cgroup/cpu.max"), "threads": {}}
        for n in (1, 2, 4, 8, 16):
            if n > len(one_per_core):
                break
            rate = run(one_per_core[:n], spp1 * n)
            out["threads"][str(n)] = {"msamples_per_s": round(rate, 3), "per_thread": round(rate / n, 4)}
            print(f"{n} threads: {rate:.3f} Msamples/s", file=sys.stderr, flush=True)
        if smt_core:
            one = run(smt_core[:1], spp1)
            two = run(smt_core[:2], 2 * spp1)
            out["smt"] = {"cpus": smt_core[:2], "one_thread": round(one, 3), "two_siblings": round(two, 3), "gain": round(two / one, 3)}
        base = out["threads"]["1"]["per_thread"]
        out["per_thread_vs_1"] = {k: round(v["per_thread"] / base, 3) for k, v in out["threads"].items()}
        print(json.dumps(out, indent=1))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
