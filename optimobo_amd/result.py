"""Result containers (optimobo/result.py:4-97): same attribute names and plot helpers."""
import numpy as np


class Res:
    """Outcome of ``solve()``: Pareto approximation, its inputs, the archive and the HV trace."""

    def __init__(self, pf_approx, pf_inputs, ysample, Xsample, hypervolume_convergence, n_obj, n_init_samples):
        self.pf_approx = pf_approx
        self.pf_inputs = pf_inputs
        self.ysample = ysample
        self.Xsample = Xsample
        self.hypervolume_convergence = hypervolume_convergence
        self.n_obj = n_obj
        self.n_init_samples = n_init_samples

    def _scatter_sets(self):
        y = np.asarray(self.ysample)
        k = self.n_init_samples
        return [(y[5:], "red", "Samples."), (np.asarray(self.pf_approx), "green", "PF approximation."),
                (y[:k], "blue", "Initial samples."), (y[-1:-5:-1], "black", "Last 5 samples.")]

    def plot_pareto_front(self):
        import matplotlib.pyplot as plt
        if self.n_obj == 2:
            for pts, colour, label in self._scatter_sets():
                plt.scatter(pts[:, 0], pts[:, 1], color=colour, label=label)
            plt.xlabel(r"$f_1(x)$")
            plt.ylabel(r"$f_2(x)$")
            plt.legend()
        elif self.n_obj == 3:
            fig, (ax1, ax2) = plt.subplots(1, 2, subplot_kw={"projection": "3d"})
            for pts, colour, label in self._scatter_sets():
                ax1.scatter(pts[:, 0], pts[:, 1], pts[:, 2], color=colour, label=label)
            pf = np.asarray(self.pf_approx)
            ax2.scatter(pf[:, 0], pf[:, 1], pf[:, 2], color="green", label="PF approximation.")
            for ax in (ax1, ax2):
                ax.set_xlabel(r"$f_1(x)$")
                ax.set_ylabel(r"$f_2(x)$")
                ax.set_zlabel(r"$f_3(x)$")
            ax1.legend()

    def plot_hv_convergence(self):
        import matplotlib.pyplot as plt
        plt.plot(self.hypervolume_convergence)


class Constrained_Res(Res):  # noqa: N801 — reference name
    """Result of the constrained optimisers, with the feasible/infeasible split."""

    def __init__(self, y_infeasible, y_feasible, X_infeasible, X_feasible, pf_approx, pf_inputs, ysample, Xsample,
                 hypervolume_convergence, n_obj, n_init_samples):
        super().__init__(pf_approx, pf_inputs, ysample, Xsample, hypervolume_convergence, n_obj, n_init_samples)
        self.X_infeasible = X_infeasible
        self.X_feasible = X_feasible
        self.y_feasible = y_feasible
        self.y_infeasible = y_infeasible
