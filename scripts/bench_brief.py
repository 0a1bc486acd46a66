#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (the headline, every config's roofline with its
in-run and rocprof launch averages, the LML / predict / build legs).

    python scripts/bench_brief.py gpurun_out/r04a/bench.json
"""
import json
import sys


def line_of(path):
    # gloo's connection messages can share stdout with the JSON line
    return json.loads([ln for ln in open(path) if ln.startswith('{"metric"')][-1])


def roof(r):
    if not r:
        return "-"
    p = r.get("rocprof") or {}
    return (f"frac {r.get('frac') or 0:.3f} inrun {r.get('avg_launch_us') or 0:.1f} us rocprof "
            f"{p.get('avg_us', 0):.1f} us ({p.get('source')})")


def main():
    d = line_of(sys.argv[1])
    print(f"C3 {d['value']} fits/s, {d['ms_per_step']} ms/step, {roof(d['roofline'])}")
    for k, v in (d.get("configs") or {}).items():
        print(f"{k} {v.get('value')} {v.get('error') or ''} {roof(v.get('roofline'))}")
    lml, pr, b = d.get("lml_grad") or {}, d.get("predict") or {}, d.get("build") or {}
    print(f"lml {lml.get('ms_wall')} ms {lml.get('phases_ms')}")
    print(f"predict {pr.get('pts_per_s_device')} pts/s tree frac {(pr.get('roofline_tree') or {}).get('frac')}")
    print(f"build {b.get('ms')} ms {b.get('gbs')} GB/s tree frac {(b.get('roofline_tree') or {}).get('frac')}")
    print(f"dist_error {d.get('dist_error')} replicas {(d.get('replicas') or {}).get('value')}")
    if d.get("ranks"):
        print(f"n_gpus {d.get('n_gpus')} ranks_seen {d.get('ranks_seen')} devices {d.get('distinct_devices')} "
              f"launcher {d.get('launcher')} transport {d.get('dist_transport')}")
        for r in d["ranks"]:
            print("  rank", {k: r.get(k) for k in ("rank", "device", "pci", "transport", "rccl_count", "push_linv",
                                                   "push_tiles", "push_bytes", "chain_step_us_median",
                                                   "diag_steps_owned", "traced_fit_ms_factor", "error")})


if __name__ == "__main__":
    main()
