"""Precision flags of inference_partition.py against the reference CLI
(/root/reference/inference_partition.py:345: --fp16 = autocast float16 during sampling / decoding).
The MI355X build has no float16 kernels: --fp16 selects the bf16 path and says so on stderr;
--bf16 names that path directly; the default stays the fp32 parity path."""
import inference_partition as ip


def test_default_is_fp32_parity_path():
    a = ip.parse_args(["--input", "x"])
    assert not a.bf16 and not a.fp16


def test_bf16_flag():
    a = ip.parse_args(["--input", "x", "--bf16"])
    assert a.bf16 and not a.fp16


def test_fp16_selects_bf16_with_notice(capsys):
    a = ip.parse_args(["--input", "x", "--fp16"])
    assert a.bf16 and a.fp16
    err = capsys.readouterr().err
    assert "--fp16" in err and "bf16" in err
