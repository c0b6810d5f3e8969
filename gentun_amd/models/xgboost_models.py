"""``XgboostModel`` -- reference-compatible GBDT k-fold CV fitness.

Reference: gentun/models/xgboost_models.py:11-37 (``xgb.DMatrix`` +
``xgb.cv`` with early stopping; returns ``test-<metric>-mean`` of the last
(best) row). xgboost is not available here, so the boosting runs on this
package's own engine (:mod:`gentun_amd.models.gbdt`): native C++ on the CPU
and HIP histogram / split kernels on MI355X.
"""

from .generic_models import GentunModel


class XgboostModel(GentunModel):

    def __init__(self, x_train, y_train, hyperparameters, booster='gbtree', objective='reg:linear',
                 eval_metric='rmse', nfold=5, num_boost_round=5000, early_stopping_rounds=100,
                 device=None, seed=0):
        super(XgboostModel, self).__init__(x_train, y_train)
        self.params = {'booster': booster, 'objective': objective, 'eval_metric': eval_metric, 'silent': 1}
        self.params.update(hyperparameters)
        self.eval_metric = eval_metric
        self.nfold = nfold
        self.num_boost_round = num_boost_round
        self.early_stopping_rounds = early_stopping_rounds
        self.device = device
        self.seed = seed
        self.history = None

    def cross_validate(self):
        from . import gbdt
        hist = gbdt.cv(self.params, self.x_train, self.y_train, num_boost_round=self.num_boost_round,
                       nfold=self.nfold, early_stopping_rounds=self.early_stopping_rounds, seed=self.seed,
                       device=self.device)
        self.history = hist
        return float(hist['test-{}-mean'.format(self.eval_metric)][-1])
