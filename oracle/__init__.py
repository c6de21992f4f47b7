"""CPU oracle for the WAM attribution hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in here is shipped or measured as the product. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the
checker (or, for ``cpu_baseline``, as the timed CPU restatement of the reference algorithm).
The product path (``wam_amd``) never imports this package and fails loudly if its HIP library is
missing.

Contents
--------
dwt.py        numpy float64 restatement of the ptwt DWT rules the reference calls
              (``lib/wam_2D.py:96,113,430``; ``lib/wam_1D.py:109,117,370``;
              ``lib/wam_3D.py:194,206,222,620``): padding per mode, stride-2 analysis, transposed
              synthesis with ptwt's crop/adjust rule, and the adjoint (zero-mode analysis).
ptwt_torch.py torch-CPU (conv/conv_transpose + autograd) restatement of the same ptwt rules with a
              ptwt-shaped API (``wavedec2``/``waverec2``/... + ``constants.WaveletDetailTuple2d``).
              This is the algorithm the reference actually executes on the CPU.
wam_ref.py    restatement of the reference glue (``BaseWAM{1,2,3}D`` / ``WaveletAttribution{1,2,3}D``)
              on top of ``ptwt_torch``: legacy numpy noise stream, mosaic, normalisation, SmoothGrad /
              IG accumulation, 3D cube and legacy averaging.
melspec.py    restatement of torchaudio's MelSpectrogram + AmplitudeToDB defaults (1D front-end).

Pinning
-------
* ``dwt.py`` and ``ptwt_torch.py`` are pinned against PyWavelets 1.1.1 known answers
  (``tests/golden/pywt_dwt.npz``) and MATLAB R2012a single-level answers shipped in pywt's test
  data (``tests/golden/matlab_dwt.npz``); generator ``tests/golden/make_pywt_fixtures.py``.
  ptwt itself (the reference's dependency) is absent offline: parity for the ptwt boundary is
  pinned through pywt, ptwt's own equality target.
* ``wam_ref.py`` is pinned against goldens produced by importing the reference's own
  ``lib/wam_{1,2,3}D.py`` in this container with ``ptwt := oracle.ptwt_torch`` and a
  ``cv2.resize`` stand-in (``tests/golden/make_glue_goldens.py``).
* ``melspec.py`` is parity-unpinned (neither torchaudio nor librosa exists offline).
"""
