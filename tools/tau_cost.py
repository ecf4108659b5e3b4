"""What the r06 refinement margins cost on natural frames (VERDICT r05 item 5:
"report the natural-frame flag rate and the call time at each new tau_N").

For N = 2, 4, 8 on the bench's 16384^2 natural-like RGB frame and N = 16 on
8192^2, at the r05 margin (4e-6 for every N) and at the r06 default
(default_tie_tau(N): 4e-6, 4e-6, 2e-5, 5e-5): pixels flagged for the fp64
refinement (host entry point, dcte_last_refined), and device times -- map
launch alone (HIP events around it, DCTE_OPT_PROFILE) and the whole call,
map + refinement (HIP events on the stream), best of 3 rounds of 10.
One JSON line per (N, tau).

    python tools/tau_cost.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dct-carver_amd")]

DEFAULT = {2: 4e-6, 4: 4e-6, 8: 2e-5, 16: 5e-5}


def main():
    import torch
    import dctenergy
    from dctenergy import synth
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    stream = st.cuda_stream
    with dctenergy.Context(ngpus=1) as ctx:
        for n in (2, 4, 8, 16):
            S = 8192 if n == 16 else 16384
            fr = synth.natural_rows(0, S, S, 3, seed=0, device=dev)
            host = fr.cpu().numpy()
            out = torch.empty((S, S), dtype=torch.float32, device=dev)
            for label, tau in (("r05 margin", 4e-6), ("r06 default", -1)):
                ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, tau)

                def call():
                    ctx.energy_map_device(fr.data_ptr(), fr.stride(0), S, S, 3, 0, S, 0, S, n, 0.3, 0.7,
                                          out.data_ptr(), out.stride(0), stream)
                for _ in range(3):
                    call()
                torch.cuda.synchronize()
                best_call, best_map = 1e9, 1e9
                for _ in range(3):
                    ctx.profile_read()
                    ctx.set_option(dctenergy.DCTE_OPT_PROFILE, 1)
                    a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a0.record(st)
                    for _ in range(10):
                        call()
                    a1.record(st)
                    torch.cuda.synchronize()
                    ctx.set_option(dctenergy.DCTE_OPT_PROFILE, 0)
                    launches, kms = ctx.profile_read()
                    best_call = min(best_call, a0.elapsed_time(a1) / 10)
                    best_map = min(best_map, kms / max(1, launches))
                ctx.energy_map(host, n, 0.3, 0.7)
                flagged = int(ctx.last_refined)
                print(json.dumps({"n": n, "size": S, "tau": tau if tau >= 0 else DEFAULT[n], "margin": label,
                                  "flagged": flagged, "flagged_per_mpx": round(flagged / (S * S / 1e6), 2),
                                  "map_ms": round(best_map, 4), "call_ms": round(best_call, 4),
                                  "refinement_ms": round(best_call - best_map, 4)}), flush=True)
            ctx.set_option(dctenergy.DCTE_OPT_TIE_TAU, -1)
            del fr, out, host
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
