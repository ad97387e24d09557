"""How long does learning that ONE tiny kernel finished take, by wait method?  (Bench
only: tools/variants sosxv_sync_probe.)  Feeds the small-message path's choice of wait
(DESIGN section 7)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants"))


def main():
    import torch
    import variants as V
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    names = ["hipStreamSynchronize", "hipStreamQuery spin", "hipEventSynchronize",
             "host spin on a flag the kernel stores",
             "one hipStreamQuery, then host spin on the flag",
             "hipStreamQuery of an idle stream alone (no launch)",
             "host spin on a flag stored relaxed (no release fence)",
             "host spin on the flag, 1024-thread workgroup"]
    out = {}
    for _ in range(2):
        for m, name in enumerate(names):
            out[name] = round(V.sync_probe(m, 2000, s.cuda_stream), 2)
    svc = {}
    for n in (1, 64, 1024, 4096):
        svc[n] = round(V.service_probe(n, 2000, s.cuda_stream), 2)
    print(json.dumps({"us_per_launch_and_wait": out,
                      "persistent_kernel_round_trip_us_by_n": svc}))


if __name__ == "__main__":
    main()
