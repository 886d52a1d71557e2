import sys; sys.path.insert(0, '.')
import torch, petershirleyraytracer_amd as P
ctx = P.Context(0)
sph = P.scene_random_spheres(1); cam = P.camera_look_at(aspect=1.5)
ctx.set_scene(sph, cam)
acc = torch.zeros((800,1200,3), dtype=torch.float64, device='cuda:0')
rgb = torch.zeros((800,1200,3), dtype=torch.uint8, device='cuda:0')
s = torch.cuda.current_stream()
for i in range(3):
    ctx.render_device(P.params(1200, 800, 100), acc.data_ptr(), rgb.data_ptr(), s.cuda_stream)
    print(ctx.sync_stats(), float(acc.sum()), flush=True)
a, r, st = P.render(sph, cam, 120, 80, 8)
print(st)
