"""Fill / drain analysis of k_even from the diagnostic per-workgroup stamps.

Build:   tools/build_variant.sh stamps "-DPSGD_EVEN_STAMPS" psgd_product_f32.hip psgd_product_bf16.hip
Run:     PSGD_LIB_PATH=powersgd_amd/_lib_v/stamps/libpsgd.so PSGD_EVEN_STAMPS=gpurun_out/st.txt \\
             python tools/step_trace.py cfg2_resnet50_r1 12
Report:  python tools/even_stamps.py gpurun_out/st.txt [skip]

Per launch (s_memrealtime, 100 MHz = 10 ns ticks): the span from the first workgroup's entry
to the last workgroup's last segment; how late workgroups enter (fill); how early they finish
relative to the last (drain); per-workgroup streaming rate; the time of each segment against
its bytes (the per-segment fixed cost)."""
import statistics
import sys

TICK_US = 0.01


def parse(path):
    for line in open(path):
        f = line.split()
        if not f:
            continue
        nwg = int(f[0])
        wgs = []
        for tok in f[1:1 + nwg]:
            parts = tok.split(":")
            nseg, byts = int(parts[0]), int(parts[1])
            st = [int(x) for x in parts[2:]]
            wgs.append((nseg, byts, st))
        yield wgs


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]


def report(wgs):
    live = [w for w in wgs if w[0] > 0 and w[2][0] > 0]
    t0 = min(w[2][0] for w in live)
    ends, starts, rates, seg_rows = [], [], [], []
    for nseg, byts, st in live:
        segs = [x for x in st[1:1 + min(nseg, 6)] if x]
        end = segs[-1] if segs else st[0]
        starts.append((st[0] - t0) * TICK_US)
        ends.append((end - t0) * TICK_US)
        dur = (end - st[0]) * TICK_US
        if dur > 0:
            rates.append(byts / dur / 1e3)  # GB/s per workgroup
        prev = st[0]
        for x in segs:
            seg_rows.append((x - prev) * TICK_US)
            prev = x
    span = max(ends)
    tot = sum(w[1] for w in live)
    print(f"workgroups {len(live)}  span {span:.2f} us  bytes {tot / 1e6:.1f} MB -> {tot / span / 1e6:.2f} TB/s")
    print(f"  entry (fill): p50 {pct(starts, .5):.2f}  p90 {pct(starts, .9):.2f}  max {max(starts):.2f} us")
    print(f"  finish: min {min(ends):.2f}  p10 {pct(ends, .1):.2f}  p50 {pct(ends, .5):.2f}  p90 {pct(ends, .9):.2f}  "
          f"max {span:.2f} us  (drain after p50: {span - pct(ends, .5):.2f} us)")
    print(f"  per-workgroup rate GB/s: p10 {pct(rates, .1):.1f}  p50 {pct(rates, .5):.1f}  p90 {pct(rates, .9):.1f}")
    nseg = [w[0] for w in live]
    print(f"  segments per workgroup: mean {statistics.mean(nseg):.2f}  max {max(nseg)}")
    # busy fraction: sum of workgroup active time / (span * resident slots)
    act = sum(e - s for s, e in zip(starts, ends))
    print(f"  sum of workgroup active time {act:.0f} us; over the span that is {act / span:.0f} workgroups resident on average")


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    launches = list(parse(path))
    for i, wgs in enumerate(launches[skip:]):
        print(f"== launch {i + skip}")
        report(wgs)


if __name__ == "__main__":
    main()
