"""Kernel reads of host memory by allocation kind (bench only, tools/variants): GB/s of
one kernel reading a buffer the host has just rewritten, and how many words it saw
stale.  Feeds the small host-resident path's choice of slot memory."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants"))


def main():
    import torch
    import variants as V
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    kinds = ["hipHostMalloc coherent", "hipHostMalloc non-coherent",
             "hipHostRegister fine-grained (small path today)", "hipHostRegister coarse-grained"]
    out = {}
    for m, k in enumerate(kinds):
        out[k] = {str(b >> 10) + " KiB": V.host_read_probe(m, b, 20, s.cuda_stream)
                  for b in (64 << 10, 1 << 20, 16 << 20)}
    print(json.dumps({"gbps_and_stale_words": out}))


if __name__ == "__main__":
    main()
