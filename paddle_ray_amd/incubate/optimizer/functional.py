"""minimize_bfgs / minimize_lbfgs (parity: python/paddle/incubate/optimizer/functional/
{bfgs,lbfgs}.py). Return (is_converge, num_func_calls, position, objective_value,
objective_gradient[, inverse_hessian_estimate]) like the reference."""
import torch
from torch.optim.lbfgs import _strong_wolfe

from ...framework.core import Tensor, _u


def _value_and_grad(f, x):
    x = x.detach().requires_grad_(True)
    with torch.enable_grad():
        v = _u(f(Tensor(x)))
        g, = torch.autograd.grad(v, x)
    return v.detach(), g.detach()


def _line_search(f, x, v, g, d, t0, max_ls, line_search_fn):
    calls = [0]

    def obj(xk, t, dk):
        calls[0] += 1
        fv, gv = _value_and_grad(f, xk + t * dk)
        return float(fv), gv
    if line_search_fn == 'strong_wolfe':
        fnew, gnew, t, _ = _strong_wolfe(obj, x, t0, d, float(v), g, float(g.dot(d)),
                                         max_ls=max_ls)
        return torch.as_tensor(fnew, dtype=x.dtype, device=x.device), gnew, t, calls[0]
    raise NotImplementedError("line_search_fn must be 'strong_wolfe'")


def minimize_bfgs(objective_func, initial_position, max_iters=50, tolerance_grad=1e-7,
                  tolerance_change=1e-9, initial_inverse_hessian_estimate=None,
                  line_search_fn='strong_wolfe', max_line_search_iters=50,
                  initial_step_length=1.0, dtype='float32', name=None):
    dt = torch.float64 if str(dtype).endswith('64') else torch.float32
    x = _u(initial_position).detach().to(dt).reshape(-1)
    n = x.numel()
    H = (torch.eye(n, dtype=dt, device=x.device) if initial_inverse_hessian_estimate is None
         else _u(initial_inverse_hessian_estimate).to(dt))
    v, g = _value_and_grad(objective_func, x)
    calls, converged = 1, False
    for _ in range(max_iters):
        if g.abs().max() <= tolerance_grad:
            converged = True
            break
        d = -H @ g
        vn, gn, t, c = _line_search(objective_func, x, v, g, d, initial_step_length,
                                    max_line_search_iters, line_search_fn)
        calls += c
        s = t * d
        x = x + s
        y = gn - g
        if (vn - v).abs() < tolerance_change or s.abs().max() < tolerance_change:
            v, g = vn, gn
            converged = True
            break
        ys = y.dot(s)
        if ys > 1e-10:
            rho = 1.0 / ys
            I = torch.eye(n, dtype=dt, device=x.device)
            A = I - rho * torch.outer(s, y)
            H = A @ H @ A.t() + rho * torch.outer(s, s)
        v, g = vn, gn
    return (Tensor(torch.tensor(converged)), Tensor(torch.tensor(calls)), Tensor(x),
            Tensor(v), Tensor(g), Tensor(H))


def minimize_lbfgs(objective_func, initial_position, history_size=100, max_iters=50,
                   tolerance_grad=1e-8, tolerance_change=1e-8,
                   initial_inverse_hessian_estimate=None, line_search_fn='strong_wolfe',
                   max_line_search_iters=50, initial_step_length=1.0, dtype='float32',
                   name=None):
    dt = torch.float64 if str(dtype).endswith('64') else torch.float32
    x = _u(initial_position).detach().to(dt).reshape(-1)
    H0 = None if initial_inverse_hessian_estimate is None else \
        _u(initial_inverse_hessian_estimate).to(dt)
    v, g = _value_and_grad(objective_func, x)
    calls, converged = 1, False
    S, Y = [], []
    for _ in range(max_iters):
        if g.abs().max() <= tolerance_grad:
            converged = True
            break
        q = g.clone()
        alphas = []
        for s, y in reversed(list(zip(S, Y))):
            a = s.dot(q) / y.dot(s)
            alphas.append(a)
            q = q - a * y
        if H0 is not None:
            r = H0 @ q
        elif S:
            r = q * (S[-1].dot(Y[-1]) / Y[-1].dot(Y[-1]))
        else:
            r = q
        for (s, y), a in zip(zip(S, Y), reversed(alphas)):
            b = y.dot(r) / y.dot(s)
            r = r + s * (a - b)
        d = -r
        vn, gn, t, c = _line_search(objective_func, x, v, g, d, initial_step_length,
                                    max_line_search_iters, line_search_fn)
        calls += c
        s = t * d
        x = x + s
        y = gn - g
        if y.dot(s) > 1e-10:
            S.append(s)
            Y.append(y)
            if len(S) > history_size:
                S.pop(0)
                Y.pop(0)
        done = (vn - v).abs() < tolerance_change or s.abs().max() < tolerance_change
        v, g = vn, gn
        if done:
            converged = True
            break
    return (Tensor(torch.tensor(converged)), Tensor(torch.tensor(calls)), Tensor(x),
            Tensor(v), Tensor(g))
