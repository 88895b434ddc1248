"""Child process of test_gpu_parity.py::test_stream_disorder_falls_back: loads the test build of
the library (KMHG_LIB_VARIANT=test -> libkmhgpu_test.so, the only build that reads
KMHG_TEST_DISORDER) and, for bucket-id and packed key streams and disorder modes 1-3, checks that
the corrupted build is detected and rebuilt by the global-atomic build with oracle-equal results.
Prints one "ok <stream> <mode>" line per case; any failure raises (non-zero exit)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    assert os.environ.get("KMHG_LIB_VARIANT") == "test", "run with KMHG_LIB_VARIANT=test"
    import torch
    from kmer_hasher_amd import _lib, synth
    from kmer_hasher_amd.device import DeviceIndex
    from test_gpu_parity import _check_against_oracle
    assert _lib.LIB_PATH.endswith("libkmhgpu_test.so"), _lib.LIB_PATH
    torch.cuda.set_device(0)
    s = synth.add_n_runs(synth.iid(300_000, 51), 0.002, 9).tobytes().decode("latin-1")
    seq = torch.frombuffer(bytearray(s.encode("latin-1")), dtype=torch.uint8).cuda()
    for stream in ("bid", "keys"):
        os.environ["KMHG_BUILD_BID"] = "1" if stream == "bid" else "0"
        for mode in ("1", "2", "3"):
            for disorder, one_bucket in (("0", False), (mode, True)):
                os.environ["KMHG_TEST_DISORDER"] = disorder
                idx = DeviceIndex.build(seq, 31).wait()
                meta, _ = idx.export_image()
                nb = int(meta[2].item()) >> 32
                assert (nb == 1) == one_bucket, (stream, disorder, nb)
                info = idx.info()          # the rebuild is reported (kmhg_info.fallback / build)
                assert info["fallback"] == (1 if one_bucket else 0), (stream, disorder, info)
                assert info["build"] == (_lib.KMHG_BUILD_GLOBAL if one_bucket else
                                         _lib.KMHG_BUILD_PARTITIONED), (stream, disorder, info)
                idx.free()
                _check_against_oracle(s, 31, pairs=False)
            print("ok", stream, mode, flush=True)
    os.environ.pop("KMHG_TEST_DISORDER", None)


if __name__ == "__main__":
    main()
