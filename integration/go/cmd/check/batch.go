package check

import (
	"bufio"
	"fmt"
	"io"
	"os"
	"strings"
	"sync"

	"github.com/ory/x/cmdx"
	"github.com/spf13/cobra"

	acl "github.com/ory/keto/proto/ory/keto/acl/v1alpha1"

	"github.com/ory/keto/cmd/client"
)

const (
	FlagBatch       = "batch"
	FlagConcurrency = "concurrency"
)

// Batch mode of `keto check` (cmd/check/root.go:27-70; the reference takes exactly 4 args, :32):
//
//	keto check --batch requests.tsv [-d max-depth] [--concurrency 256]
//	keto check --batch - < requests.tsv
//
// Each input line is `<subject> <relation> <namespace> <object>` separated by tabs (or, when a
// line has no tab, by single spaces).  Requests go over one gRPC connection as concurrent
// CheckService.Check calls, so the server's micro-batcher (internal/gpu/batcher.go) coalesces them
// into GPU batches; no new RPC is needed.  Output: one Allowed / Denied line per request, in input
// order (checkOutput, root.go:16-23).  Register with
//
//	cmd.Flags().String(FlagBatch, "", "file of `subject relation namespace object` lines, - for stdin")
//	cmd.Flags().Int(FlagConcurrency, 256, "concurrent Check calls in batch mode")
//
// and, in newCheckCmd, replace `Args: cobra.ExactArgs(4)` with `Args: checkArgs` and start RunE with
//
//	if f, _ := cmd.Flags().GetString(FlagBatch); f != "" {
//		return runBatch(cmd, f)
//	}
func checkArgs(cmd *cobra.Command, args []string) error {
	if f, _ := cmd.Flags().GetString(FlagBatch); f != "" {
		return cobra.NoArgs(cmd, args)
	}
	return cobra.ExactArgs(4)(cmd, args)
}

type batchReq struct {
	subject, relation, namespace, object string
}

func readBatch(r io.Reader) ([]batchReq, error) {
	var out []batchReq
	sc := bufio.NewScanner(r)
	sc.Buffer(make([]byte, 1<<16), 1<<20)
	for line := 1; sc.Scan(); line++ {
		t := sc.Text()
		if strings.TrimSpace(t) == "" {
			continue
		}
		sep := "\t"
		if !strings.Contains(t, "\t") {
			sep = " "
		}
		f := strings.Split(t, sep)
		if len(f) != 4 {
			return nil, fmt.Errorf("line %d: want 4 fields <subject> <relation> <namespace> <object>, got %d", line, len(f))
		}
		out = append(out, batchReq{f[0], f[1], f[2], f[3]})
	}
	return out, sc.Err()
}

func runBatch(cmd *cobra.Command, file string) error {
	in := cmd.InOrStdin()
	if file != "-" {
		f, err := os.Open(file)
		if err != nil {
			return err
		}
		defer f.Close()
		in = f
	}
	reqs, err := readBatch(in)
	if err != nil {
		return err
	}
	maxDepth, err := cmd.Flags().GetInt32(FlagMaxDepth)
	if err != nil {
		return err
	}
	workers, err := cmd.Flags().GetInt(FlagConcurrency)
	if err != nil {
		return err
	}
	if workers < 1 {
		workers = 1
	}
	conn, err := client.GetReadConn(cmd)
	if err != nil {
		return err
	}
	defer conn.Close()
	cl := acl.NewCheckServiceClient(conn)

	allowed := make([]bool, len(reqs))
	errs := make([]error, len(reqs))
	next := make(chan int)
	var wg sync.WaitGroup
	for w := 0; w < workers; w++ {
		wg.Add(1)
		go func() {
			defer wg.Done()
			for i := range next {
				r := reqs[i]
				resp, err := cl.Check(cmd.Context(), &acl.CheckRequest{
					Subject:   &acl.Subject{Ref: &acl.Subject_Id{Id: r.subject}},
					Relation:  r.relation,
					Namespace: r.namespace,
					Object:    r.object,
					MaxDepth:  maxDepth,
				})
				if err != nil {
					errs[i] = err
					continue
				}
				allowed[i] = resp.Allowed
			}
		}()
	}
	for i := range reqs {
		next <- i
	}
	close(next)
	wg.Wait()
	for i := range reqs {
		if errs[i] != nil {
			_, _ = fmt.Fprintf(cmd.ErrOrStderr(), "Could not make request %d: %s\n", i+1, errs[i])
			return errs[i]
		}
		cmdx.PrintJSONAble(cmd, &checkOutput{Allowed: allowed[i]})
	}
	return nil
}
