import sys, os, ctypes
sys.path.insert(0, '.')
import numpy as np
import vkcomputeshader_tinyraytracer_amd as trt
from vkcomputeshader_tinyraytracer_amd import scene as S
sc = S.config_reference_default(env_size=(1024, 512), width=int(sys.argv[1]), height=int(sys.argv[2]))
r = trt.Renderer(0)
r.upload_scene(sc)
r.set_deferred_shadows(2)
r.set_subtree_split(int(sys.argv[3]))
a8, _, _ = r.draw_frame(sc.params())
print("stages", os.environ.get("TRT_DEFER_STAGES"), "ok", r.defer_stats(0), flush=True)
L = trt.lib()
out = (ctypes.c_uint32 * 16)()
L.trt_diag_defer_pad.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
L.trt_diag_defer_pad(r._h, 0, out)
print("pad", list(out), flush=True)
r.set_deferred_shadows(1)
r.set_subtree_split(1)
b8, _, _ = r.draw_frame(sc.params())
d = np.abs(a8.astype(int) - b8.astype(int)).max(-1)
ys, xs = np.nonzero(d)
print("diff px", len(ys), list(zip(ys[:10].tolist(), xs[:10].tolist())), flush=True)
