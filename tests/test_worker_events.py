"""WorkerHandle::recv_event's verdict on non-gradient frames, on the CPU
(ono_worker_event_check is host code of the product library; the TCP ring
calls the same function, tests/test_gpu_tcp.py checks it end to end).

Reference: comms/src/handles/worker.rs:82-130 (recv_event),
comms/src/protocol/msg.rs:41-88 (Command: serde, externally tagged,
snake_case), :160-191 (Msg::deserialize), :194-229 (null losses -> NaN),
worker/src/middlewares/worker_ring.rs:136-138, 195-197 (the ring rejects any
event that is not a gradient).  Parity of the serde messages themselves is
unpinned (serde_json is not in the image): the classes and the reference's own
strings ("Received an invalid worker event", "loss diverged: NaN or Inf
detected", "Unexpected message from worker", "Received an invalid kind byte")
are what the tests fix.
"""
import pytest

import ono_amd

PROTO, IO = ono_amd.InvalidWorkerEvent, ono_amd.IoError


@pytest.mark.parametrize("kind", [1, 2, 3, 4])
def test_gradients_pass(kind):
    ono_amd.worker_event_check(kind, b"\0\0")


@pytest.mark.parametrize("payload", [b'"upgraded"', b'"disconnect"', b'"done"', b' {"done" : null} ',
                                     b'{"upgraded":null}', b'{"report_loss":{"losses":[]}}',
                                     b'{"report_loss":{"losses":[0.5,-1e-3,2E+2]}}',
                                     b'{"report_loss":{"losses":[1],"extra":{"a":[true,false]}}}',
                                     b'{"report_loss":[[1.5, 2]]}'])
def test_worker_events_the_ring_rejects(payload):
    """Upgraded / Disconnect / Done / a finite ReportLoss are WorkerEvents;
    the ring's `let WorkerEvent::Grad {..} = event else` turns them into
    "Received an invalid worker event" (worker_ring.rs:136-138)."""
    with pytest.raises(PROTO, match="Received an invalid worker event"):
        ono_amd.worker_event_check(0, payload)


@pytest.mark.parametrize("payload", [b'{"report_loss":{"losses":[null]}}', b'{"report_loss":{"losses":[1,null,2]}}',
                                     b'{"report_loss":[[null]]}'])
def test_nan_loss_diverged(payload):
    """null deserializes as NaN (msg.rs:201-229); recv_event refuses a
    non-finite loss (worker.rs:113-115)."""
    with pytest.raises(IO, match="loss diverged: NaN or Inf detected"):
        ono_amd.worker_event_check(0, payload)


@pytest.mark.parametrize("payload", [b'"ping"', b'"pong"', b'"eof"', b'"request_params"', b'"share_dataset"',
                                     b'"stop_after_epoch"', b'{"connect":{"id":"0","src":"worker"}}',
                                     b'{"accept":{}}', b'{"share_dataset_size":{"size":1}}', b'{"switch":[]}'])
def test_other_commands_unexpected(payload):
    """Any other command reaches recv_event's `msg =>` arm (worker.rs:123-126)."""
    with pytest.raises(IO, match="Unexpected message from worker"):
        ono_amd.worker_event_check(0, payload)


@pytest.mark.parametrize("kind", [5, 6])
def test_params_and_datachunks_unexpected(kind):
    with pytest.raises(IO, match="Unexpected message from worker"):
        ono_amd.worker_event_check(kind, b"\0" * 8)


@pytest.mark.parametrize("payload", [b"", b"   ", b"nul", b'"done', b'"done" "done"', b"[1,]", b'{"a":1,}',
                                     b'{"done":null,"upgraded":null}', b"01", b"1.", b"-", b'"\\x"', b'"\x01"',
                                     b'"\\ud800"', b'"\xff"', b'{"report_loss":{"losses":[1e999]}}',
                                     b'{"report_loss":{}}', b'{"report_loss":{"losses":1}}',
                                     b'{"report_loss":{"losses":["a"]}}', b'{"report_loss":{"losses":[1],"losses":[2]}}',
                                     b'"report_loss"', b'{"done":1}', b'{"bogus":null}', b"[]", b"3",
                                     b"[" * 200 + b"]" * 200, b'{"connect":1}'])
def test_serde_errors(payload):
    """Malformed JSON, unknown commands and ill-typed payloads are the serde
    error that `serde_json::from_slice(rest)?` turns into an io::Error (msg.rs:171)."""
    with pytest.raises(IO):
        ono_amd.worker_event_check(0, payload)


@pytest.mark.parametrize("kind", [7, 8, 100, 255])
def test_invalid_kind_byte(kind):
    with pytest.raises(IO, match=f"Received an invalid kind byte {kind}"):
        ono_amd.worker_event_check(kind, b"")


def test_unicode_and_escapes_parse():
    ono_amd.worker_event_check(1, b"")
    with pytest.raises(PROTO):  # a valid command after escaped / multi-byte key content elsewhere
        ono_amd.worker_event_check(0, '{"report_loss":{"losses":[1],"k\\u00e9\\ud83d\\ude00é":"\\n\\t"}}'.encode())
