"""CPU oracle for the MADDPG training hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain numpy/Python restatement of the reference
(adolfogonzalez3/maddpg, mounted read-only at /root/reference during the
build) and of the third-party code its hot path calls:

* ``pyrandom``  -- CPython's MT19937 + ``random.randint`` rejection sampling
  (the module-global RNG used by ``replay_buffer.py:46-47``).
* ``replay``    -- ``maddpg/trainer/replay_buffer.py:5-85``.
* ``nets``      -- ``experiments/train.py:39-46`` (mlp_model), TF1 ops used by
  ``maddpg/trainer/maddpg.py`` (Gumbel-softmax ``distributions.py:264-266``,
  ``tf_util.minimize_and_clip`` ``tf_util.py:166-182``, TF1 ``ApplyAdam``,
  the Polyak update ``maddpg.py:20-26``).
* ``trainer``   -- ``MADDPGAgentTrainer.update`` (``maddpg.py:161-196``).
* ``mpe``       -- the multiagent-particle-envs scenarios used by
  ``experiments/train.py:48-61`` (third-party, NOT vendored in the reference;
  restated from its published source, version unpinned).
* ``train_loop`` -- ``experiments/train.py:78-189`` call structure, used as
  the timed CPU baseline (``cpu_baseline.kind == "port"``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker or the
baseline being timed -- never as the product path.  The product path
(``maddpg_amd``) runs on the HIP library and fails loudly when it is missing.

Parity pinning (see DESIGN.md "Oracle"):
* replay index selection + gather: PINNED against golden fixtures generated
  by importing the reference's own ``ReplayBuffer`` (``tests/golden/``).
* trainer math: parity vs TF1 UNPINNED (TensorFlow is not importable here and
  no reference test covers ``maddpg/trainer/maddpg.py``); restated op by op.
* MPE physics: parity UNPINNED (MPE is absent from the container and the
  reference pins no test at that boundary).
"""
