"""CPU oracle for the DL4SS separation hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain numpy / torch-CPU restatement of the reference algorithm
(shincling/DL4SS, Python-2 / torch-0.3 research code that cannot be imported or run
here).  It exists only to *check* the HIP path:

* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
  leg may import it;
* nothing under ``dl4ss_amd/`` imports it, and the product path never falls back
  to it.

Parity status: the reference ships no golden vectors, known-answer tests or
fixtures for this path.  Each oracle function is pinned
instead against in-container independent references (``numpy.fft``, ``torch.nn.LSTM``
/ ``torch.nn.GRU`` on CPU, closed-form identities: Parseval, STFT->iSTFT perfect
reconstruction, MSE gradients) -- see ``tests/test_oracle.py``.  librosa is not
installed and its version is unpinned by the reference, so the STFT convention
(librosa >= 0.6: periodic Hann, centre/reflect padding, no conjugation) is a
documented choice; ``conj=True`` restates librosa 0.5.x.
"""
