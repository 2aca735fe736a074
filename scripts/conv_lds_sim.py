"""CPU check of enc_conv_nhwc_kernel's plane-major LDS images (csrc/ggd_encoder.hip CGeo): for every
compiled tile shape, (1) every MFMA operand read addresses the patch position the convolution needs,
(2) the LDS cycles of each ds_read_b128 (patch and filter) and ds_write_b128 (patch) wave instruction
under MI355X_MICROARCH.md's lane groups (4 / 8 = conflict-free).  python3 scripts/conv_lds_sim.py"""
import itertools
groups=[[0,1,2,3,12,13,14,15]+list(range(20,28)),[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
groups+= [[l+32 for l in g] for g in groups]
wgroups=[list(range(8*i,8*i+8)) for i in range(8)]
def cyc(addrs, gs):
    tot=0
    for g in gs:
        banks={}
        for l in g:
            a=addrs[l]
            for d in range(4): banks.setdefault(((a//4)+d)%64,set()).add(a//4+d)
        tot+=max(len(s) for s in banks.values())
    return tot
def geo(TW,KS,ST):
    TH=128//TW
    PH= TH if KS==1 else (TH-1)*ST+KS
    PW= TW if KS==1 else (TW-1)*ST+KS
    PS= 1 if KS==1 else ST
    SS= ST if KS==1 else 1
    DI= KS>1 and ST==2
    HALF=(PW+1)//2
    PWC= 2*HALF if DI else PW
    w=PWC
    if TW==8:
        while (PS*w)%16!=8: w+=1
    PWS=w
    NPOS=(PH*PWS+15)//16*16
    TAPS=KS*KS; TAPSP=TAPS|1
    col=lambda px: (px&1)*HALF+(px>>1) if DI else px
    return dict(TH=TH,PH=PH,PW=PW,PS=PS,SS=SS,DI=DI,HALF=HALF,PWS=PWS,NPOS=NPOS,TAPS=TAPS,TAPSP=TAPSP,col=col)
for (NJ,TW,KS,ST) in [(2,16,3,1),(4,16,3,1),(4,8,3,1),(4,16,3,2),(4,8,3,2),(4,16,1,2),(4,8,1,2),(4,16,2,1),(2,16,3,1)]:
    G=geo(TW,KS,ST)
    pad = 1 if KS==3 else 0
    NP=G['NPOS']*4
    # staging map: LDS element offset (pos,q) -> patch coord (py,px) or None
    lds={}
    for v in range(NP):
        p=(v>>5)*8+(v&7); q=(v>>3)&3
        py=p//G['PWS']; pc=p%G['PWS']
        px=(2*pc if pc<G['HALF'] else 2*(pc-G['HALF'])+1) if G['DI'] else pc
        key=(q,p)
        assert key not in lds
        lds[key]=(py,px) if (py<G['PH'] and px<G['PW']) else None
    assert len(lds)==NP
    # reads: every wave, tile i, lane, tap
    bad=0; rc=[]; 
    for wave in range(4):
        for i in range(2):
            for tap in range(G['TAPS']):
                ky,kx=tap//KS,tap%KS
                toff=ky*G['PWS']+G['col'](kx)
                addrs=[]
                for lane in range(64):
                    r16,g=lane&15,lane>>4
                    qq=wave*32+i*16+r16; ty,tx=qq//TW,qq%TW
                    pos=ty*G['PS']*G['PWS']+tx+toff
                    got=lds.get((g,pos),'missing')
                    want=(ty*(G['PS'] if KS>1 else 1)+ky, tx*(G['PS'] if KS>1 else 1)+kx) if KS>1 else (ty,tx)
                    if got!=want: bad+=1
                    addrs.append((g*G['NPOS']+pos)*16)
                rc.append(cyc(addrs,groups))
    # weight reads
    NWQ=NJ*16*G['TAPSP']; wc=[]
    for tap in range(G['TAPS']):
        for j in range(NJ):
            addrs=[((lane>>4)*NWQ+(j*16+(lane&15))*G['TAPSP']+tap)*16 for lane in range(64)]
            wc.append(cyc(addrs,groups))
    # patch writes
    pw=[]
    for k in range((NP+255)//256):
        for wave in range(4):
            addrs=[]
            for lane in range(64):
                v=min(wave*64+lane+k*256,NP-1)
                p=(v>>5)*8+(v&7); q=(v>>3)&3
                addrs.append((q*G['NPOS']+p)*16)
            pw.append(cyc(addrs,wgroups))
    lds_kb=(G['NPOS']*64+4*NWQ*16)/1024
    print((NJ,TW,KS,ST),"bad",bad,"patch read cyc",max(rc),"w read",max(wc),"patch write",max(pw),"LDS KB %.1f"%lds_kb)
