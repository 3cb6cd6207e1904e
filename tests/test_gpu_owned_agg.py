"""The owned aggregation (EBD_AGG=own: k_own_count, k_own_emit, k_own_part, k_own; the service
table in 2048-slot ranges, each one workgroup's, in LDS) through the parity cases that create
services: every outcome and the service table compared with the oracle bit for bit.  It is an
alternative to k_agg_fast, measured slower, kept exact by these cases."""
import pytest

import test_gpu_parity as P

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def owned_path(monkeypatch):
    monkeypatch.setenv("EBD_AGG", "own")


def test_aggregator_vectors_real_checker(vectors):
    P.test_aggregator_vectors_real_checker(vectors)


@pytest.mark.parametrize("align", [1, 16])
def test_config3_sample_single_and_multi_batch(align):
    P.test_config3_sample_single_and_multi_batch(align)


def test_fragmented_keepalive_sessions():
    P.test_fragmented_keepalive_sessions()


def test_large_config3_against_oracle():
    P.test_large_config3_against_oracle()


def test_clear_and_resubmit_creates_each_service_once():
    P.test_clear_and_resubmit_creates_each_service_once()


def test_client_ip_queue_drains_every_request():
    P.test_client_ip_queue_drains_every_request()


def test_device_export_by_owner_and_merge_equals_whole_trace():
    P.test_device_export_by_owner_and_merge_equals_whole_trace()
