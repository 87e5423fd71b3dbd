"""CPU checks of the PVCNN.models mirror: the reference configs' import line
resolves against it, and the sph-dg / cu-dg models build with the
reference's module tree (state_dict keys) -- no GPU launch."""
import pytest


def test_config_import_line_resolves():
    # configs/modelnet40/pvcnn/__init__.py:1, verbatim
    from PVCNN.models.pvcnn_classify import PVCNN_classifier
    import PVCNN.models as models
    assert PVCNN_classifier is models.pvcnn_classify.PVCNN_classifier
    from PVCNN.models.utils import create_mlp_components, create_pointnet_components  # noqa


def _sph_dg(**kw):
    from PVCNN.models.pvcnn_classify import PVCNN_classifier
    args = dict(blocks=((64, 1, 32), (128, 1, 32), (256, 1, None), (512, 1, None)), dim_k=512,
                point_kernel_formal="dgcnn_kernel", voxel_shape="spherical", num_classes=40,
                extra_feature_channels=0, rot_invariant_preprocess="change_coords",
                with_local_feat="ppf", use_new_coords_for_voxel=False, with_coeff=True,
                with_se=True)
    args.update(kw)
    return PVCNN_classifier(**args)


def test_sph_dg_module_tree():
    m = _sph_dg()
    keys = set(m.state_dict())
    # first PVConv: 3 change_coords channels + 64 fused local-PPF channels
    assert m.in_channels == 67
    for k in ("fuser.layers.0.weight", "fuser.layers.3.weight",
              "point_features.0.coefficient",
              "point_features.0.voxel_layers.0.weight",
              "point_features.0.voxel_layers.6.fc.0.weight",
              "point_features.0.point_layers.layers.0.weight",
              "point_features.2.layers.0.weight",
              "classifier.0.0.weight", "classifier.0.1.running_mean",
              "classifier.2.0.weight", "classifier.3.weight"):
        assert k in keys, k
    assert tuple(m.point_features[0].voxel_layers[0].weight.shape) == (64, 67, 3, 3, 3)
    assert tuple(m.point_features[0].point_layers.layers[0].weight.shape) == (64, 134, 1)
    assert tuple(m.classifier[3].weight.shape) == (40, 256)


def test_cu_dg_module_tree():
    m = _sph_dg(voxel_shape="cube", extra_feature_channels=4, with_coeff=False,
                is_classify=False)
    assert m.in_channels == 71
    assert not hasattr(m.point_features[0], "coefficient")


def test_unsupported_options_raise_like_reference():
    m = _sph_dg(with_local_feat="change_coords")
    assert not hasattr(m, "fuser")
    with pytest.raises(AssertionError):
        _sph_dg(rot_invariant_preprocess="ppf", extra_feature_channels=0)
