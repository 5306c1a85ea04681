import sys, numpy as np, torch
sys.path.insert(0, '.')
import tcp_amd
dev = torch.device("cuda:0")
payload = torch.empty(1 << 26, dtype=torch.uint8, device=dev)
tcp_amd.synth_fill(payload, 0, payload.numel())
def build(offs, tl, rb):
    m = offs.size
    segs = np.zeros(m, tcp_amd.TXSEG_DTYPE)
    segs["payload_off"] = (np.arange(m, dtype=np.uint64) * 4096) % np.uint64(payload.numel() - 65536)
    segs["out_off"] = offs
    segs["saddr_be"], segs["daddr_be"] = 0x0100007F, np.arange(m, dtype=np.uint32)
    segs["sport"], segs["dport"], segs["len"], segs["flags"] = 4000, 45001, tl - 24, 1 | 16
    reg = torch.zeros(rb, dtype=torch.uint8, device=dev)
    tcp_amd.tx_build(payload, torch.from_numpy(segs.view(np.uint8)).to(dev), m, int(tl.max()), reg, 0, None)
    return reg
for n in (4096, 65536, 1 << 20):
    offs = np.arange(n, dtype=np.uint64) * 1536
    reg = build(offs, np.full(n, 1480, np.uint32), n * 1536)
    doff = torch.from_numpy(offs.view(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev); sta = torch.empty(n, dtype=torch.uint8, device=dev)
    base = reg.clone()
    tcp_amd.ipv4_batch(reg, doff, n, 1536, 0, out, sta)
    a_out, a_reg, a_st = out.clone(), reg.clone(), sta.clone()
    reg.copy_(base)
    tcp_amd.ipv4_batch(reg, doff, n, 1536, 0, out, sta, tune=tcp_amd.make_tuning(0, 0, -1, 512))
    torch.cuda.synchronize()
    print(n, "out eq", torch.equal(a_out, out), "st eq", torch.equal(a_st, sta), "reg eq", torch.equal(a_reg, reg),
          "status0", int((a_st == 0).sum()), "base ptr mod 128", reg.data_ptr() % 128)
    if not torch.equal(a_reg, reg):
        d = (a_reg != reg).nonzero().flatten().cpu().numpy()
        print(" first diffs", d[:10], "count", d.size, "slot offs", np.unique(d % 1536)[:20])
        i = int(d[0]) // 1536
        print(" pkt", i, "u16", a_reg[i*1536:i*1536+64].cpu().numpy(), "\n line", reg[i*1536:i*1536+64].cpu().numpy(),
              "\n base", base[i*1536:i*1536+64].cpu().numpy())
    if not torch.equal(a_out, out):
        d = (a_out != out).nonzero().flatten().cpu().numpy()
        print(" out diffs", d[:10], d.size)
    del reg, base, a_reg
    torch.cuda.empty_cache()
# A/B order: the line FILL over packets the u16 FILL already filled
for n in (4096, 1 << 20):
    offs = np.arange(n, dtype=np.uint64) * 1536
    reg = build(offs, np.full(n, 1480, np.uint32), n * 1536)
    doff = torch.from_numpy(offs.view(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev); sta = torch.empty(n, dtype=torch.uint8, device=dev)
    tcp_amd.ipv4_batch(reg, doff, n, 1536, 0, out, sta)
    a_out, a_reg = out.clone(), reg.clone()
    tcp_amd.ipv4_batch(reg, doff, n, 1536, 0, out, sta, tune=tcp_amd.make_tuning(0, 0, -1, 512))
    torch.cuda.synchronize()
    print("refill", n, "out eq", torch.equal(a_out, out), "reg eq", torch.equal(a_reg, reg))
    if not torch.equal(a_reg, reg):
        d = (a_reg != reg).nonzero().flatten().cpu().numpy()
        print(" first diffs", d[:10], "count", d.size, "slot offs", np.unique(d % 1536)[:20])
    tcp_amd.ipv4_batch(reg, doff, n, 1536, 1, out, sta)
    torch.cuda.synchronize()
    print(" verify zero", bool((out == 0).all().item()), bool((sta == 0).all().item()), int((out != 0).sum().item()))
    if not torch.equal(a_out, out):
        pass
    del reg, a_reg
    torch.cuda.empty_cache()
