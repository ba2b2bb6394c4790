"""Fit and check the fp32 sin/cos of nerf_device.h sincos_acc (CPU only).

    python tools/sincos_lab.py

Fits minimax-like polynomials (relative least squares on Chebyshev nodes, float64)
for sin and cos on [-pi/4, pi/4], then emulates the kernel's fp32 arithmetic
(3-part Cody-Waite reduction by pi/2 with FMA, Horner with FMA; numpy float64
products rounded to float32) over the reference encoding's arguments
fl(fl(2^k pi) x), k < 10, |x| <= 10.5, and reports the distance to torch's CPU
sin / cos (what PositionalEncoding.encode calls, nerf.py:41-43) in ulps.
"""
import numpy as np, torch
f32=np.float32
def fma(a,b,c): return f32(np.float64(a)*np.float64(b)+np.float64(c))
P1=f32(np.pi/2); P2=f32(np.pi/2-np.float64(P1)); P3=f32(np.pi/2-np.float64(P1)-np.float64(P2))
TWO_OVER_PI=f32(2/np.pi)
# fit polynomials in float64 (near-minimax via Chebyshev-node least squares, relative)
xs=np.cos(np.linspace(0,np.pi,4001))*(np.pi/4*1.02)
xs=xs[np.abs(xs)>1e-6]
z=xs*xs
def fit(deg, target, w):
    A=np.stack([z**i for i in range(deg+1)],1)
    c,*_=np.linalg.lstsq(A*w[:,None], target*w, rcond=None)
    return c
# sin(x) = x + x*z*(s0 + s1 z + s2 z^2 + ...)
def fit_sin(n):
    t=(np.sin(xs)-xs)/(xs*z); w=np.abs(xs*z)/np.abs(np.sin(xs))
    return fit(n,t,w)
def fit_cos(n):
    t=(np.cos(xs)-1+0.5*z)/(z*z); w=(z*z)/np.abs(np.cos(xs))
    return fit(n,t,w)
def sincos32(a, S, C):
    a=f32(a)
    q=f32(np.rint(f32(a*TWO_OVER_PI)))
    r=fma(-q,P1,a); r=fma(-q,P2,r); r=fma(-q,P3,r)
    zz=f32(r*r)
    ps=f32(S[-1])
    for c in S[-2::-1]: ps=fma(ps,zz,f32(c))
    s=fma(f32(r*zz),ps,r)
    pc=f32(C[-1])
    for c in C[-2::-1]: pc=fma(pc,zz,f32(c))
    co=fma(f32(zz*zz),pc,fma(f32(-0.5),zz,f32(1.0)))
    qi=int(q)&3
    if qi==0: return s,co
    if qi==1: return co,-s
    if qi==2: return -s,-co
    return -co,s
rng=np.random.RandomState(0)
x=np.concatenate([rng.uniform(-2,2,3000),rng.uniform(-10.5,10.5,3000)]).astype(np.float32)
args=[]
for k in range(10):
    c=f32(np.float32(2.0**k)*np.float32(np.pi))
    args.append((c*x).astype(np.float32))
args=np.concatenate(args)
ts=torch.sin(torch.from_numpy(args)).numpy(); tc=torch.cos(torch.from_numpy(args)).numpy()
def ulps(a,b):
    ia=a.view(np.int32).astype(np.int64); ib=b.view(np.int32).astype(np.int64)
    ia=np.where(ia<0, -2**31-ia, ia); ib=np.where(ib<0,-2**31-ib,ib)
    return np.abs(ia-ib)
for ns,nc in [(2,2),(3,3),(3,4),(4,4)]:
    S=fit_sin(ns); C=fit_cos(nc)
    S32=[f32(v) for v in S]; C32=[f32(v) for v in C]
    sub=args[::7]
    res=np.array([sincos32(a,S32,C32) for a in sub],dtype=np.float32)
    us=ulps(res[:,0],ts[::7]); uc=ulps(res[:,1],tc[::7])
    ds=np.abs(res[:,0]-ts[::7]).max(); dc=np.abs(res[:,1]-tc[::7]).max()
    print(ns,nc,'sin ulps max',us.max(),'p99.9',np.percentile(us,99.9),'cos ulps max',uc.max(), 'abs',ds,dc, [float(v) for v in S32],[float(v) for v in C32])
