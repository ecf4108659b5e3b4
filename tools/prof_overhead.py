"""Cost of DCTE_OPT_PROFILE's launch-recorded events on the step time: the
bench's 16384^2 N = 8 step (one map + refinement launch) and a strong-scaling
rank's 2048-row band step (interior launch + one two-range edge launch, as
bench.py at world 8), timed on the stream with the events off and on,
interleaved, best of 5 rounds of 50 steps.  One JSON line per case.

    python tools/prof_overhead.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]


def main():
    import torch
    import dctenergy
    from dctenergy import synth
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    s = st.cuda_stream
    W, n = 16384, 8
    with dctenergy.Context(ngpus=1) as ctx:
        fr = synth.natural_rows(0, W, W, 3, seed=0, device=dev)
        out = torch.empty((W, W), dtype=torch.float32, device=dev)
        hl, hr = n // 2 - 1, n // 2
        R = 2048
        Y0, Y1 = 3 * R, 4 * R

        def full():
            ctx.energy_map_device(fr.data_ptr(), fr.stride(0), W, W, 3, 0, W, 0, W, n, 0.3, 0.7,
                                  out.data_ptr(), out.stride(0), s)

        def band():
            ctx.energy_map_device(fr.data_ptr(), fr.stride(0), W, W, 3, 0, W, Y0 + hl, Y1 - hr, n, 0.3, 0.7,
                                  out[Y0 + hl:].data_ptr(), out.stride(0), s)
            ctx.energy_map_device2(fr.data_ptr(), fr.stride(0), W, W, 3, 0, W, Y0, Y0 + hl, Y1 - hr, Y1,
                                   n, 0.3, 0.7, out[Y0:].data_ptr(), out.stride(0), s)
        for name, step in (("16384^2 step", full), ("2048-row band step (interior + edges)", band)):
            best = {0: 1e9, 1: 1e9}
            for _ in range(5):
                for prof in (0, 1):
                    ctx.profile_read()
                    ctx.set_option(dctenergy.DCTE_OPT_PROFILE, prof)
                    for _ in range(5):
                        step()
                    a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a0.record(st)
                    for _ in range(50):
                        step()
                    a1.record(st)
                    torch.cuda.synchronize()
                    ctx.set_option(dctenergy.DCTE_OPT_PROFILE, 0)
                    ctx.profile_read()
                    best[prof] = min(best[prof], a0.elapsed_time(a1) / 50)
            print(json.dumps({"case": name, "ms_per_step_events_off": round(best[0], 4),
                              "ms_per_step_events_on": round(best[1], 4),
                              "overhead_us": round((best[1] - best[0]) * 1e3, 2),
                              "overhead_frac": round(best[1] / best[0] - 1, 4)}), flush=True)


if __name__ == "__main__":
    main()
