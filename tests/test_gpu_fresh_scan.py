"""The structural scan (k_fresh_scan, EBD_CFG_FRESH_SCAN: lanes over pieces, header lines and
buffers of an LDS tile, ebd_scan.h) through the parity cases the DFA kernel (k_fresh) runs:
every outcome compared with the oracle bit for bit.  EBD_FRESH=scan selects it for each
context the cases create."""
import pytest

import test_gpu_parity as P

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def scan_path(monkeypatch):
    monkeypatch.setenv("EBD_FRESH", "scan")


def test_config1_probe(vectors):
    P.test_config1_probe(vectors)


def test_reference_parser_vectors_as_sessions(vectors):
    P.test_reference_parser_vectors_as_sessions(vectors)


def test_reference_parser_vectors_interleaved_and_closed(vectors):
    P.test_reference_parser_vectors_interleaved_and_closed(vectors)


def test_aggregator_vectors_real_checker(vectors):
    P.test_aggregator_vectors_real_checker(vectors)


def test_checker_vectors_through_the_path(vectors):
    P.test_checker_vectors_through_the_path(vectors)


@pytest.mark.parametrize("align", [1, 16])
def test_config3_sample_single_and_multi_batch(align):
    P.test_config3_sample_single_and_multi_batch(align)


def test_config2_sample():
    P.test_config2_sample()


def test_fragmented_keepalive_sessions():
    P.test_fragmented_keepalive_sessions()


def test_missing_buffers_and_data_end_only():
    P.test_missing_buffers_and_data_end_only()


def test_large_config3_against_oracle():
    P.test_large_config3_against_oracle()


def test_config4_fragmented_keepalive_parity_1m():
    P.test_config4_fragmented_keepalive_parity_1m(4)
