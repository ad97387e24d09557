"""One PE of test_gpu_fakerccl.test_init_attr_multi_pe: shmemx_get_unique_id on PE 0, the
id handed to the other PEs out of band (a file, as a launcher would broadcast it), then
shmemx_init_attr -- no TCP bootstrap and no node shared memory, so barriers are RCCL's and
team agreement (split_strided) goes through the RCCL team-word exchange.  Then it runs
tests/team_check_pe.py or tools/team_mgmt_check.py (argv[1]) on top of that runtime.

Environment: INIT_ATTR_PE, INIT_ATTR_NPES, INIT_ATTR_UID_FILE.
"""
import os
import runpy
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

from sos_amd import shmem as S  # noqa: E402


def init_from_uid():
    me, n = int(os.environ["INIT_ATTR_PE"]), int(os.environ["INIT_ATTR_NPES"])
    path = os.environ["INIT_ATTR_UID_FILE"]
    if me == 0:
        uid = S.get_unique_id()
        with open(path + ".part", "wb") as f:
            f.write(uid)
        os.rename(path + ".part", path)
    else:
        t0 = time.time()
        while not os.path.exists(path):
            if time.time() - t0 > 60:
                raise TimeoutError("no unique id from PE 0")
            time.sleep(0.01)
        with open(path, "rb") as f:
            uid = f.read()
    S.init_attr(me, n, uid)


if __name__ == "__main__":
    S.shmem_init = init_from_uid
    sys.argv = sys.argv[1:]
    runpy.run_path(sys.argv[0], run_name="__main__")
