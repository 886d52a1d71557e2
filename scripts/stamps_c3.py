"""Diagnostic: C3 section clocks of the stamps kernel variant (stderr)."""
import sys, os; sys.path.insert(0, '.')
import torch, petershirleyraytracer_amd as P
ctx = P.Context(0)
sph = P.scene_random_spheres(1); cam = P.camera_look_at(aspect=1.5)
ctx.set_scene(sph, cam)
acc = torch.zeros((800,1200,3), dtype=torch.float64, device='cuda:0')
s = torch.cuda.current_stream()
ctx.render_device(P.params(1200, 800, 100), acc.data_ptr(), 0, s.cuda_stream); ctx.sync_stats()
ctx.set_tuning('stamps', 1)  # the diagnostic kernel variant (include/rt.h tuning knobs)
ctx.render_device(P.params(1200, 800, 100), acc.data_ptr(), 0, s.cuda_stream); print(ctx.sync_stats(), flush=True)
