import sys, time
sys.path.insert(0, '.')
from xraytracer_amd import scenes
from xraytracer_amd.renderer import HipRenderer
import torch
cfg = scenes.CONFIGS['C4']
s = scenes.build('C4')
r = HipRenderer(64, device=0)
r.upload(s)
W, H = cfg['width'], cfg['height']
fb = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda:0')
st = r.render_device(s, W, H, fb.data_ptr())
torch.cuda.synchronize()
print('segments', st.segments, 'shadow', st.shadow_rays, 'samples', st.samples, 'iters', st.iterations)
