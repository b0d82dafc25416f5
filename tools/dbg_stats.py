"""Print the pool kernel's per-wave diagnostic counters for one render."""
import argparse, json, os, sys
os.environ["RTP_DEBUG_STATS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import raytracingtherestofyourlife_amd as rtp
ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--n", type=int, default=800)
ap.add_argument("--variant", type=int, default=0)
ap.add_argument("--world", type=int, default=1, help="render rank --rank's share of the 16x16 tile deal")
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--ff-tables", default="on", choices=["on", "auto", "off"])
a = ap.parse_args()
dev = rtp.Device(0); dev.set_cornell_box(a.variant); dev.set_ff_tables(a.ff_tables)
from raytracingtherestofyourlife_amd import shard
ids = torch.from_numpy(shard.tile_pixels(a.n, a.n, a.rank, a.world)).cuda() if a.world > 1 else None
npx = a.n * a.n if ids is None else ids.numel()
out = torch.zeros((npx, 4), dtype=torch.float32, device="cuda")
live = torch.zeros(npx, dtype=torch.int32, device="cuda")
st = dev.render_device(rtp.default_camera(), a.n, a.n, a.spp, a.depth, out.data_ptr(), pixel_count=npx,
                       pixel_ids_ptr=0 if ids is None else ids.data_ptr(),
                       stream=torch.cuda.current_stream().cuda_stream, live_ptr=live.data_ptr(), timed=True)
c = dev.debug_counters()
samples = npx * a.spp
L = live.to(torch.int64).sum().item()
c.update(kernel_ms=st.kernel_ms, samples=samples, live_bounces=L,
         lanes_per_bounce_step=c["bounce_lanes"] / max(1, c["bounce_steps"]),
         lanes_per_ff=c["ff_lanes"] / max(1, c["ff_phases"]),
         ff_iters_per_phase=c["ff_iters"] / max(1, c["ff_phases"]),
         frac_cycles_ff=c["cycles_ff"] / max(1, c["cycles_total"]),
         frac_cycles_bounce=c["cycles_bounce"] / max(1, c["cycles_total"]),
         cycles_per_bounce_step=c["cycles_bounce"] / max(1, c["bounce_steps"]),
         cycles_per_ff_phase=c["cycles_ff"] / max(1, c["ff_phases"]),
         avg_wave_over_max=c["cycles_total"] / max(1, c["waves"]) / max(1, c["max_wave_cycles"]),
         per_step_intersect=c["cycles_intersect"] / max(1, c["bounce_steps"]),
         per_step_shade=(c["cycles_bounce_call"] - c["cycles_intersect"]) / max(1, c["bounce_steps"]),
         per_step_end=c["cycles_end"] / max(1, c["bounce_steps"]),
         per_step_refill=c["cycles_refill"] / max(1, c["bounce_steps"]),
         tail_frac_steps=c["tail_steps"] / max(1, c["bounce_steps"]),
         tail_lanes_per_step=c["tail_lanes"] / max(1, c["tail_steps"]),
         tail_frac_cycles=c["tail_cycles"] / max(1, c["cycles_total"]),
         fallback_frac_steps=c["fallback_steps"] / max(1, c["bounce_steps"]),
         fallback_lanes_per_step=c["fallback_lanes"] / max(1, c["bounce_steps"]))
# exec occupancy per region (round 4): lanes active at the region's start
regions = {"bounce (intersect)": ("bounce_steps", "bounce_lanes"), "surface hit (shade)": ("hit_visits", "hit_lanes"),
           "Lambertian (generator + pdfs)": ("gen_visits", "gen_lanes"), "dielectric": ("diel_visits", "diel_lanes"),
           "light hit": ("light_visits", "light_lanes"), "path end": ("end_visits", "end_lanes"),
           "refill (camera ray)": ("refill_visits", "refill_lanes"), "fast-forward batch": ("ff_phases", "ff_lanes"),
           "  radiance product": ("ffrad_visits", "ffrad_lanes"), "  hashed dead depths": ("ff_iters", "dead_lanes")}
c["regions"] = {k: {"visits": c[v], "visits_per_step": round(c[v] / max(1, c["bounce_steps"]), 4),
                    "lanes": round(c[l] / max(1, c[v]), 2)} for k, (v, l) in regions.items()}
c["regions"]["  radiance product"]["rows_per_lane"] = round(c["ffrad_rows"] / max(1, c["ffrad_lanes"]), 2)
c["per_step_gen"] = c["cycles_gen"] / max(1, c["bounce_steps"])
c["per_step_pdf"] = c["cycles_pdf"] / max(1, c["bounce_steps"])
c["per_step_diel"] = c["cycles_diel"] / max(1, c["bounce_steps"])
print(json.dumps(c, indent=1))
rec = dev.debug_wave_records()
import numpy as np
start, end = rec[:, 12].astype(np.int64), rec[:, 13].astype(np.int64)
t0 = start.min()
life = (end - start) / 100.0  # us (100 MHz)
fin = (end - t0) / 100.0
print("wave start spread us", (start.max() - t0) / 100.0, "finish us: min/p10/p50/p90/max",
      [round(float(np.percentile(fin, q)), 1) for q in (0, 10, 50, 90, 100)])
hw = rec[:, 14].astype(np.int64)
wave_id = hw & 0xF; simd = (hw >> 4) & 3; cu = (hw >> 8) & 0xF
print("lifetime by wave-in-SIMD slot:", {int(s): round(float(life[wave_id == s].mean()), 1) for s in np.unique(wave_id)})
order = np.argsort(start)
print("lifetime of earliest-started quartile vs latest:", round(float(life[order[:len(order)//4]].mean()),1), round(float(life[order[-len(order)//4:]].mean()),1))
