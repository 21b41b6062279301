"""Diagnostic: the 1-rank RCCL graph-step rehearsal of
tests/test_ops_gpu.py::_graph_comm_1rank_worker with bucket-aware weight-
gradient flushing (64-job batches), printing every row -- parameter / loss
differences graph vs eager, the reducer race probe (max |snapshot - final
gradient|: a collective that read its bucket before the last deposit) and
NaN-ness -- so the ordering fixes can be checked by switching them off
(D3D_DIAG_SINK_NO_STREAM_WAITS=1: collectives wait only for the issuing
stream, the round-5 behaviour under which the bf16 row produced NaN).

    python tools/diag_bucket_flush_race.py [out_dir]
"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from distributed_3d_diffusion_pytorch_amd.parallel import spawn
    import test_ops_gpu as t
    out = sys.argv[1] if len(sys.argv) > 1 else tempfile.mkdtemp()
    os.makedirs(out, exist_ok=True)
    spawn(t._graph_comm_1rank_worker, 1, (out, True))
    print("row  d_param  d_loss  mode  exposed  race_eager  race_graph  probed")
    print(open(os.path.join(out, "gc1.txt")).read())


if __name__ == "__main__":
    main()
