"""Find the first front-end layer whose output differs when two sub-batches run on concurrent streams
(against the same sub-batches run one after another). Diagnostic for tools/streams_ab.py."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from damvsnet_amd import frontend_hip as F
    H, W, N, nd, dtype, _ = bench.CONFIGS["cfgC"]
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    imgs, proj, dv, ins = bench.make_inputs(4, N, H, W, dev)
    chunks = [(imgs[i * 2:(i + 1) * 2], {k: v[i * 2:(i + 1) * 2] for k, v in proj.items()}, dv[i * 2:(i + 1) * 2])
              for i in range(2)]
    rec = {}
    orig = F.HipConv2d.__call__

    def spy(self, B, Hi, Wi, in0=None, in1=None, geo=(), **k):
        ins = [t.clone() for t in (in0, in1) if t is not None] + [g.clone() for g, _ in geo] + \
              [v.clone() for v in k.values() if isinstance(v, torch.Tensor)]
        out = orig(self, B, Hi, Wi, in0, in1, geo, **k)
        rec.setdefault(torch.cuda.current_stream().cuda_stream, []).append((self, out, ins))
        return out

    main_s = torch.cuda.current_stream()
    with torch.no_grad():
        net(*chunks[0])
        torch.cuda.synchronize()
        F.HipConv2d.__call__ = spy
        seq = []
        for c in chunks:
            rec.clear()
            net(*c)
            seq.append(list(rec[main_s.cuda_stream]))
        torch.cuda.synchronize()
        for trial in range(6):
            streams = [torch.cuda.Stream() for _ in range(2)]
            rec.clear()
            for st, c in zip(streams, chunks):
                st.wait_stream(main_s)
                with torch.cuda.stream(st):
                    net(*c)
            torch.cuda.synchronize()
            for i, st in enumerate(streams):
                con = rec[st.cuda_stream]
                for j, ((L, a, ia), (_, b, ib)) in enumerate(zip(con, seq[i])):
                    same_in = [torch.equal(x, y) for x, y in zip(ia, ib)]
                    if not torch.equal(a, b) or not all(same_in):
                        d = (a.float() - b.float()).abs()
                        print("trial %d chunk %d: layer #%d (%d calls) differs: %d elements, max %.3e, shape %s, "
                              "cout %d, ngeo %d; inputs equal: %s" % (trial, i, j, len(con), int((d > 0).sum()),
                                                                      d.max().item(), tuple(a.shape), L.cout, L.ngeo,
                                                                      same_in), flush=True)
                        break
                else:
                    print("trial %d chunk %d: all %d layers equal" % (trial, i, len(con)), flush=True)


if __name__ == "__main__":
    main()
