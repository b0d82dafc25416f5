"""One C2-geometry render for counter collection (rocprofv3 --pmc)."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import raytracingtherestofyourlife_amd as rtp
ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--n", type=int, default=800)
a = ap.parse_args()
dev = rtp.Device(0); dev.set_cornell_box(0)
out = torch.zeros((a.n * a.n, 4), dtype=torch.float32, device="cuda")
st = dev.render_device(rtp.default_camera(), a.n, a.n, a.spp, a.depth, out.data_ptr(),
                       stream=torch.cuda.current_stream().cuda_stream, timed=True)
print("kernel_ms", st.kernel_ms)
