"""Concurrent codec sessions (RDEIC.session(): own launch plans, pinned buffers and host state,
shared weights), one host thread + HIP stream each, as bench.py --streams runs them: every session
must produce exactly the single-session bitstreams and pixels, and a plan replayed on a stream other
than the one it was recorded on must be refused (its launches and host-step events are bound there)."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
B, S = 3, 128


def _inputs():
    from rdeic_amd.synthetic import relay_noise, synth_context, synth_image
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 500 + i) for i in range(B)])).cuda()
    noise = torch.cat([relay_noise((1, 4, S // 8, S // 8), 500 + i, 2)[0] for i in range(B)])
    return imgs, noise, synth_context().cuda()


def test_concurrent_sessions_match_single_session(gpu):
    from rdeic_amd.rdeic import RDEIC
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
    imgs, noise, ctx = _inputs()
    m.use_plans = False
    ref_out, ref_bodies = m.codec_images(imgs, ctx, noise, steps=2)  # eager, default stream
    m.use_plans = True
    sessions = [m.session() for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in sessions]
    for s, st in zip(sessions, streams):  # record one session at a time
        with torch.cuda.stream(st):
            s.codec_images(imgs, ctx, noise, steps=2)
        torch.cuda.synchronize()
    results, errors = {}, []

    def run(j):
        try:
            with torch.cuda.stream(streams[j]):
                for r in range(3):
                    out, bodies = sessions[j].codec_images(imgs, ctx, noise, steps=2)
                    torch.cuda.current_stream().synchronize()
                    results[(j, r)] = (out.cpu(), bodies)
        except BaseException as e:
            errors.append(e)

    th = [threading.Thread(target=run, args=(j,)) for j in range(len(sessions))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for (j, r), (out, bodies) in results.items():
        assert bodies == ref_bodies, (j, r)
        assert torch.equal(out, ref_out.cpu()), (j, r)
    # a session's plans are bound to the stream they were recorded on
    with torch.cuda.stream(streams[1]):
        with pytest.raises(RuntimeError, match="different stream"):
            sessions[0].codec_images(imgs, ctx, noise, steps=2)


def test_eager_sessions_in_threads_keep_entropy_split(gpu):
    """Eager (no plan) sessions on concurrent threads: the bf16 entropy nets' split-K switch is
    per thread (ops.splitk_allowed), so one session leaving its region never turns split-K off under
    another's — every thread's bitstreams and pixels equal the single-thread ones."""
    from rdeic_amd.rdeic import RDEIC
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
    m.use_plans = False
    imgs, noise, ctx = _inputs()
    ref_out, ref_bodies = m.codec_images(imgs, ctx, noise, steps=2)
    sessions = [m.session() for _ in range(3)]
    for s in sessions:
        s.use_plans = False
    streams = [torch.cuda.Stream() for _ in sessions]
    results, errors = {}, []

    def run(j):
        try:
            with torch.cuda.stream(streams[j]):
                for r in range(2):
                    out, bodies = sessions[j].codec_images(imgs, ctx, noise, steps=2)
                    torch.cuda.current_stream().synchronize()
                    results[(j, r)] = (out.cpu(), bodies)
        except BaseException as e:
            errors.append(e)

    th = [threading.Thread(target=run, args=(j,)) for j in range(len(sessions))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    assert len(results) == 6
    for (j, r), (out, bodies) in results.items():
        assert bodies == ref_bodies, (j, r)
        assert torch.equal(out, ref_out.cpu()), (j, r)
