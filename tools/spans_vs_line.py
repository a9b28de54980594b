"""The isolated-pass rocprof stage spans (tools/rocpd_stages.py output) next to
a bench line's roofline_isolated.stages_ms (HIP events around the same
stages of the same kind of batches), with the relative difference.

    python tools/spans_vs_line.py stage_spans_isolated.txt bench.json [more.json ...]
"""
import json
import sys


def main(spans_txt, *jsons):
    spans = {}
    for ln in open(spans_txt):
        p = ln.strip().split(",")
        if len(p) >= 2:
            try:
                spans[p[0]] = float(p[1])
            except ValueError:
                pass
    lines = [(j, json.load(open(j))) for j in jsons]
    print("stage,rocprof_ms," + ",".join(f"{j}_ms,{j}_diff_pct" for j, _ in lines))
    for st, ms in sorted(spans.items(), key=lambda kv: -kv[1]):
        row = [st, f"{ms:.4f}"]
        for _, d in lines:
            v = (d.get("roofline_isolated") or {}).get("stages_ms", {}).get(st)
            row += [f"{v:.4f}" if v else "", f"{100.0 * (v - ms) / ms:+.1f}" if v and ms else ""]
        print(",".join(row))


if __name__ == "__main__":
    main(*sys.argv[1:])
