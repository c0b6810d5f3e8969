#!/usr/bin/env python
"""Single GBDT model, 3-fold CV RMSE on white-wine quality
(reference tests/test_xgboost_model.py:11-24)."""
import _common

if __name__ == "__main__":
    from gentun import XgboostModel

    x, y = _common.wine()
    genes = {
        'eta': 0.3, 'min_child_weight': 1, 'max_depth': 6, 'gamma': 0.0, 'max_delta_step': 0,
        'subsample': 1.0, 'colsample_bytree': 1.0, 'colsample_bylevel': 1.0, 'lambda': 1.0,
        'alpha': 0.0, 'scale_pos_weight': 1.0
    }
    model = XgboostModel(x, y, genes, nfold=3)
    print(model.cross_validate())
