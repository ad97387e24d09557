import os, sys, json
sys.path.insert(0, os.getcwd())
import torch
from sos_amd import _lib
_lib.lib()
print("RT", json.dumps(_lib.loaded_runtimes()))
print("PRELOAD", os.environ.get("LD_PRELOAD"), os.environ.get("ROCP_TOOL_LIBRARIES"))
