"""Drop-in ``models`` package (the reference deploys its model files as ``code_80/models``,
README.md:13-19): mix_transformer_evp, segformer_head, mstcn, adapter_transformer,
transformer2_3_1, data_process.  Put this package's parent directory on sys.path (as the
reference's scripts run from code_80/) and ``import models.mix_transformer_evp`` etc."""
